#!/bin/bash
# round 4 session v: who publishes phase A's control block (VIGPATH_PUB_MODE:
# 3 the fold as before, 0 the classify's last block with fences, 1 without
# the blocks' fences, 2 also without the release) and fold deferral
# (VIGPATH_DEFER), headline kernel and step on one box
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VIGPATH_PUB_MODE=2 timeout -k 10 400 python -u -m pytest tests/test_nat_gpu.py tests/test_golden.py tests/test_mbuf_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04v_pytest.out 2>&1 || { tail -30 gpurun_out/r04v_pytest.out; exit 1; }
tail -1 gpurun_out/r04v_pytest.out
B="python3 bench.py --no-cpu --no-e2e --no-extra --steps 20"
for v in "3 0" "0 0" "1 0" "2 0" "2 1" "3 0" "2 0" "2 1"; do
  set -- $v
  VIGPATH_PUB_MODE=$1 VIGPATH_DEFER=$2 timeout -k 10 200 $B > gpurun_out/r04v_p$1d$2.out 2>&1 || exit $?
  echo "pub=$1 defer=$2 $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*' gpurun_out/r04v_p$1d$2.out | tr '\n' ' ')"
done
VIGPATH_PUB_MODE=2 VIGPATH_DEFER=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04v_kt -- $B > gpurun_out/r04v_kt.log 2>&1 || exit $?
