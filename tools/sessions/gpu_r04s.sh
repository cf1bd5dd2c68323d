#!/bin/bash
# round 4 session s: lean-tile miss slices through the LDS cursor array:
# GPU suite, churn, same-box A/B of the headline against abtmp/ (963d63c)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_session.sh r04s tests || exit $?
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/bench_extra.py nat_churn > gpurun_out/r04s_churn.out 2>&1 || exit $?
B="python3 bench.py --no-cpu --no-e2e --no-extra --steps 20"
for i in 1 2 3; do
  (cd abtmp && timeout -k 10 200 $B > ../gpurun_out/r04s_old$i.out 2>&1) || exit $?
  timeout -k 10 200 $B > gpurun_out/r04s_new$i.out 2>&1 || exit $?
done
grep -o '"value": [0-9.]*, "unit": "Mpps", "ms_per_step": [0-9.]*\|"state_match": [a-z]*' gpurun_out/r04s_churn.out
grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*' gpurun_out/r04s_old*.out gpurun_out/r04s_new*.out
