#!/bin/bash
# round 4 session af: vignat's control block after reprobes published and
# polled (no copy launch or stream query): GPU suite, random-key workload
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_session.sh r04af tests || exit $?
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 200 python3 tools/bench_extra.py nat_random_keys > gpurun_out/r04af_random$i.out 2>&1 || exit $?
  grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*' gpurun_out/r04af_random$i.out | tr '\n' ' '; echo
done
