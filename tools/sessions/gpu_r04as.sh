#!/bin/bash
# round 4 session as: the fold in the uniform order (40 us): chunks in
# flight per fold wave (VIGPATH_FOLD_U 8/16/32) and more bins
# (VIGPATH_BIN_BITS 9/10: more fold blocks, shorter bins). Fold 40 us at
# U = 8, 16, 32 alike; 51 us at 512 bins, 90 us at 1024 (more, sparser
# slices); round robin at 1024 bins 0.4935 vs 0.4767 ms. Defaults kept
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VIGPATH_BIN_BITS=10 timeout -k 10 400 python -u -m pytest tests/test_nat_gpu.py tests/test_golden.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04as_pytest.out 2>&1 || { tail -30 gpurun_out/r04as_pytest.out; exit 1; }
tail -1 gpurun_out/r04as_pytest.out
for v in "8 8" "16 8" "32 8" "8 9" "8 10" "16 10"; do
  set -- $v
  rm -rf gpurun_out/r04as_kt_$1_$2
  VIGPATH_FOLD_U=$1 VIGPATH_BIN_BITS=$2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04as_kt_$1_$2 -- python3 bench.py --order uniform --steps 10 --warmup 2 --no-cpu --no-e2e --no-extra > gpurun_out/r04as_$1_$2.log 2>&1 || exit $?
  echo "U=$1 bbits=$2 $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*' gpurun_out/r04as_$1_$2.log | tr '\n' ' ')"
done
for b in 8 10; do
  VIGPATH_BIN_BITS=$b timeout -k 10 200 python3 bench.py --no-cpu --no-e2e --no-extra --steps 20 > gpurun_out/r04as_rr_$b.log 2>&1 || exit $?
  echo "rr bbits=$b $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*' gpurun_out/r04as_rr_$b.log | tr '\n' ' ')"
done
