#!/bin/bash
# round 5 session zd: viglb with one 1024-thread block per CU
# (VIGPATH_LB_WAVES=16) -- viglb tests under it, then config4_lb A/B twice
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
VIGPATH_LB_WAVES=16 timeout -k 10 600 python -u -m pytest tests/test_lb_gpu.py tests/test_mbuf_gpu.py -x -q --timeout 200 --timeout-method thread > $O/r05zd_pytest.out 2>&1 || { tail -30 $O/r05zd_pytest.out; exit 1; }
tail -1 $O/r05zd_pytest.out
for i in 1 2; do
for w in 4 16; do
VIGPATH_LB_WAVES=$w timeout -k 10 300 python3 tools/bench_extra.py config4_lb > $O/r05zd_lb_w$w.out 2>&1 || { tail -20 $O/r05zd_lb_w$w.out; exit 1; }
tail -1 $O/r05zd_lb_w$w.out | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['config4_lb']; print('w$w', d['ms_per_step'], d['kernel_ms_per_launch'], d['frac'], d['parity']['match'])"
done
done
