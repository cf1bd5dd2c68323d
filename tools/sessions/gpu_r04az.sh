#!/bin/bash
# round 4 session az: what the touch bins cost the uniform order's classify
# (VIGPATH_TOUCH_BINS=0: the per-packet touch log and its sort-based fold).
# Classify 0.786 -> 0.625 ms without bins, step 0.832 -> 0.899 ms (the
# log fold is slower)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 1 0 1 0; do
  VIGPATH_TOUCH_BINS=$v timeout -k 10 200 python3 bench.py --order uniform --no-cpu --no-e2e --no-extra --steps 20 > gpurun_out/r04az_b$v.out 2>&1 || exit $?
  echo "bins=$v $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*' gpurun_out/r04az_b$v.out | tr '\n' ' ')"
done
