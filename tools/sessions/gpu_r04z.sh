#!/bin/bash
# round 4 session z: 128-byte slots with the next tile prefetched at two
# waves per SIMD (VIGPATH_128P=1) against the current kernel; then session
# y (owner route-all, 2-rank rehearsal). Measured slower (0.90 vs 0.88 ms), reverted
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VIGPATH_128P=1 timeout -k 10 400 python -u -m pytest tests/test_nat_gpu.py -k "wide or slot" -x -q --timeout 120 --timeout-method thread > gpurun_out/r04z_pytest.out 2>&1 || { tail -30 gpurun_out/r04z_pytest.out; exit 1; }
tail -1 gpurun_out/r04z_pytest.out
B="python3 bench.py --slot 128 --no-cpu --no-e2e --no-extra --steps 10"
for i in 1 2; do
  for pf in 0 1; do
    VIGPATH_128P=$pf timeout -k 10 200 $B > gpurun_out/r04z_s128_p${pf}_$i.out 2>&1 || exit $?
    echo "128P=$pf $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"frac": [0-9.]*' gpurun_out/r04z_s128_p${pf}_$i.out | tr '\n' ' ')"
  done
done
bash tools/sessions/gpu_r04y.sh
