#!/bin/bash
# round 4 session ak: 128-byte slots with the next tile prefetched at three
# waves per SIMD (VIGPATH_128P=3; 168 registers) and two (=2) against the
# current kernel, one box. Both slower (0.927, 0.908 vs 0.887 ms), not kept
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VIGPATH_128P=3 timeout -k 10 400 python -u -m pytest tests/test_nat_gpu.py -k "wide or slot" -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ak_pytest.out 2>&1 || { tail -30 gpurun_out/r04ak_pytest.out; exit 1; }
tail -1 gpurun_out/r04ak_pytest.out
B="python3 bench.py --slot 128 --no-cpu --no-e2e --no-extra --steps 10"
for pf in 0 3 2 0 3 2; do
  VIGPATH_128P=$pf timeout -k 10 200 $B > gpurun_out/r04ak_p$pf.out 2>&1 || exit $?
  echo "128P=$pf $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"frac": [0-9.]*\|"match": [a-z]*' gpurun_out/r04ak_p$pf.out | tr '\n' ' ')"
done
