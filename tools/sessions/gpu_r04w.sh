#!/bin/bash
# round 4 session w: run words in a per-block row ([block][bin], whole
# lines) instead of 64 bin entries per round-robin wave: GPU suite, same-box
# A/B (VIGPATH_BIN_RUNS=0/1, and abtmp/ = 963d63c), kernel trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_session.sh r04w tests || exit $?
export TMPDIR=/tmp
B="python3 bench.py --no-cpu --no-e2e --no-extra --steps 20"
for i in 1 2; do
  (cd abtmp && timeout -k 10 200 $B > ../gpurun_out/r04w_old$i.out 2>&1) || exit $?
  VIGPATH_BIN_RUNS=0 timeout -k 10 200 $B > gpurun_out/r04w_r0_$i.out 2>&1 || exit $?
  VIGPATH_BIN_RUNS=1 timeout -k 10 200 $B > gpurun_out/r04w_r1_$i.out 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04w_kt -- $B > gpurun_out/r04w_kt.log 2>&1 || exit $?
for f in gpurun_out/r04w_old*.out gpurun_out/r04w_r*.out; do echo "$f $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*' $f | tr '\n' ' ')"; done
