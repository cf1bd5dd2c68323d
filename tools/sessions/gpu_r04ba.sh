#!/bin/bash
# round 4 session ba: fewer touch bins (VIGPATH_BIN_BITS 6, 7 against 8):
# uniform order (its bin entries leave a block's 256 slices' lines partly
# written in the L2s) and round robin; vignat tests at 64 bins
# (run with VIGPATH_BIN_BITS accepting 6..10, a build not kept). Uniform
# classify 0.786 -> 0.748 / 0.711 ms; round-robin step 0.474 -> 0.488 /
# 0.520 ms (fewer, larger fold blocks)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VIGPATH_BIN_BITS=6 timeout -k 10 400 python -u -m pytest tests/test_nat_gpu.py tests/test_golden.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ba_pytest.out 2>&1 || { tail -30 gpurun_out/r04ba_pytest.out; exit 1; }
tail -1 gpurun_out/r04ba_pytest.out
for b in 8 7 6 8 7 6; do
  VIGPATH_BIN_BITS=$b timeout -k 10 200 python3 bench.py --order uniform --no-cpu --no-e2e --no-extra --steps 20 > gpurun_out/r04ba_u$b.out 2>&1 || exit $?
  VIGPATH_BIN_BITS=$b timeout -k 10 200 python3 bench.py --no-cpu --no-e2e --no-extra --steps 20 > gpurun_out/r04ba_r$b.out 2>&1 || exit $?
  echo "bbits=$b uniform $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*' gpurun_out/r04ba_u$b.out | tr '\n' ' ') rr $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*' gpurun_out/r04ba_r$b.out | tr '\n' ' ')"
done
