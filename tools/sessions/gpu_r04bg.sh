#!/bin/bash
# round 4 session bg: one fold block per bin at 128 bins (VIGPATH_FOLD_SPLIT=0:
# each entry read once, half the fold blocks) against two per bin (default)
# Same within noise (rr 0.4734-0.4752 vs 0.4720-0.4748 ms, uniform
# 0.8096-0.8138 vs 0.8116-0.8142); the switch was not kept
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VIGPATH_FOLD_SPLIT=0 timeout -k 10 400 python -u -m pytest tests/test_nat_gpu.py tests/test_golden.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04bg_pytest.out 2>&1 || { tail -30 gpurun_out/r04bg_pytest.out; exit 1; }
tail -1 gpurun_out/r04bg_pytest.out
for v in 1 0 1 0 1 0; do
  VIGPATH_FOLD_SPLIT=$v timeout -k 10 200 python3 bench.py --no-cpu --no-e2e --no-extra --steps 20 > gpurun_out/r04bg_r$v.out 2>&1 || exit $?
  VIGPATH_FOLD_SPLIT=$v timeout -k 10 200 python3 bench.py --order uniform --no-cpu --no-e2e --no-extra --steps 20 > gpurun_out/r04bg_u$v.out 2>&1 || exit $?
  echo "split=$v rr $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*' gpurun_out/r04bg_r$v.out | tr '\n' ' ') | uni $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*' gpurun_out/r04bg_u$v.out | tr '\n' ' ')"
done
