#!/bin/bash
# round 4 session ai: the raised issue priority as the default (lean tile of
# every vignat classify kernel); A/B against VIGPATH_PRIO=0 at 64- and
# 128-byte slots, one box; vignat GPU tests under the default
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_nat_gpu.py tests/test_golden.py tests/test_mbuf_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ai_pytest.out 2>&1 || { tail -30 gpurun_out/r04ai_pytest.out; exit 1; }
tail -1 gpurun_out/r04ai_pytest.out
for sl in 64 128; do
  B="python3 bench.py --no-cpu --no-e2e --no-extra --steps 20 --slot $sl"
  for v in 0 1 0 1 0 1; do
    VIGPATH_PRIO=$v timeout -k 10 200 $B > gpurun_out/r04ai_s${sl}p$v.out 2>&1 || exit $?
    echo "slot=$sl prio=$v $(grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"frac": [0-9.]*\|"match": [a-z]*' gpurun_out/r04ai_s${sl}p$v.out | tr '\n' ' ')"
  done
done
