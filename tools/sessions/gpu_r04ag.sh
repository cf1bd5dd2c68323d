#!/bin/bash
# round 4 session ag: vignat's lean tile with its hash and row-request issue
# at a raised wave priority (VIGPATH_PRIO=1) against the default, one box
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VIGPATH_PRIO=1 timeout -k 10 400 python -u -m pytest tests/test_nat_gpu.py tests/test_golden.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ag_pytest.out 2>&1 || { tail -30 gpurun_out/r04ag_pytest.out; exit 1; }
tail -1 gpurun_out/r04ag_pytest.out
B="python3 bench.py --no-cpu --no-e2e --no-extra --steps 20"
for v in 0 1 0 1 0 1; do
  VIGPATH_PRIO=$v timeout -k 10 200 $B > gpurun_out/r04ag_p$v.out 2>&1 || exit $?
  echo "prio=$v $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*' gpurun_out/r04ag_p$v.out | tr '\n' ' ')"
done
