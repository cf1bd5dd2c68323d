#!/bin/bash
# round 4 session u: deferred folds (a steady batch's fold runs with the next
# batch's; the classify's last block publishes the control block): GPU
# suite, same-box A/B of the headline against abtmp/ (963d63c), churn
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_session.sh r04u tests || exit $?
export TMPDIR=/tmp
B="python3 bench.py --no-cpu --no-e2e --no-extra --steps 20"
for i in 1 2 3; do
  (cd abtmp && timeout -k 10 200 $B > ../gpurun_out/r04u_old$i.out 2>&1) || exit $?
  timeout -k 10 200 $B > gpurun_out/r04u_new$i.out 2>&1 || exit $?
done
timeout -k 10 200 python3 tools/bench_extra.py nat_churn > gpurun_out/r04u_churn.out 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04u_kt -- $B > gpurun_out/r04u_kt.log 2>&1 || exit $?
grep -o '"value": [0-9.]*, "unit": "Mpps", "ms_per_step": [0-9.]*\|"state_match": [a-z]*' gpurun_out/r04u_churn.out
grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*' gpurun_out/r04u_old*.out gpurun_out/r04u_new*.out
