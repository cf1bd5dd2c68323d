#!/bin/bash
# round 4 session r: same-box A/B of the headline kernel, the tree before the
# per-block miss slices (abtmp/, commit 963d63c) against the current one
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --no-cpu --no-e2e --no-extra --steps 20"
for i in 1 2 3; do
  (cd abtmp && timeout -k 10 200 $B > ../gpurun_out/r04r_old$i.out 2>&1) || exit $?
  timeout -k 10 200 $B > gpurun_out/r04r_new$i.out 2>&1 || exit $?
done
grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*' gpurun_out/r04r_*.out
