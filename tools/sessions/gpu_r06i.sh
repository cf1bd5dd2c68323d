#!/bin/bash
# round 6 session i: vigbridge on one 1024-thread block per CU
# (VIGPATH_BRIDGE_WAVES=16) -- the bridge tests at 16 waves, then config 3
# and config 4 (viglb, VIGPATH_LB_WAVES) at 4 and 16 waves, interleaved twice
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
VIGPATH_BRIDGE_WAVES=16 timeout -k 10 600 python -u -m pytest tests/test_bridge_gpu.py tests/test_spec_gpu.py tests/test_golden.py -x -q \
  --timeout 200 --timeout-method thread -k "bridge" > $O/r06i_pytest.log 2>&1 || { tail -40 $O/r06i_pytest.log; exit 1; }
tail -1 $O/r06i_pytest.log
for i in 1 2; do
for w in 4 16; do
  VIGPATH_BRIDGE_WAVES=$w timeout -k 10 300 python3 tools/bench_extra.py config3_bridge > $O/r06i_br_$w.json 2> $O/r06i_br_$w.err || { tail -20 $O/r06i_br_$w.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['config3_bridge']
print(sys.argv[2], d['value'], d['ms_per_step'], d['kernel'], d['kernel_ms_per_launch'], d['parity']['match'])" $O/r06i_br_$w.json "bridge w$w"
  VIGPATH_LB_WAVES=$w timeout -k 10 300 python3 tools/bench_extra.py config4_lb > $O/r06i_lb_$w.json 2> $O/r06i_lb_$w.err || { tail -20 $O/r06i_lb_$w.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['config4_lb']
print(sys.argv[2], d['value'], d['ms_per_step'], d['kernel'], d['kernel_ms_per_launch'], d['parity']['match'])" $O/r06i_lb_$w.json "lb w$w"
done
done
