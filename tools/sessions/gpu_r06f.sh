#!/bin/bash
# round 6 session f: the pipelined vignat tiles with LDS-DMA rows
# (nat_tiles_pipe; VIGPATH_PIPE=12: 768-thread blocks, 168 VGPRs; 16: 1024
# threads, which spill) -- vignat tests at 12, then an A/B against the
# default tiles: round robin, uniform order, random keys
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
VIGPATH_PIPE=12 timeout -k 10 600 python -u -m pytest tests/test_nat_gpu.py tests/test_golden.py \
  tests/test_layout_gpu.py tests/test_spec_gpu.py -x -q --timeout 200 --timeout-method thread \
  > $O/r06f_pipe12.log 2>&1 || { tail -30 $O/r06f_pipe12.log; exit 1; }
tail -1 $O/r06f_pipe12.log
for i in 1 2; do
for order in rr uniform; do
for pw in 0 12 16; do
  VIGPATH_PIPE=$pw timeout -k 10 300 python3 bench.py --order $order --no-cpu --no-e2e --no-extra --steps 10 \
    > $O/r06f_ab_${order}_$pw.json 2> $O/r06f_ab_${order}_$pw.err || { tail -20 $O/r06f_ab_${order}_$pw.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print(sys.argv[2], d['value'], d['ms_per_step'], r['kernel'], r['kernel_ms_per_launch'], r.get('shape_ceiling_ms'), r.get('kernel_over_ceiling'))" $O/r06f_ab_${order}_$pw.json "$order pipe=$pw"
done
done
for pw in 0 12; do
  VIGPATH_PIPE=$pw timeout -k 10 300 python3 tools/bench_extra.py nat_random_keys > $O/r06f_rk_$pw.json 2> $O/r06f_rk_$pw.err || { tail -20 $O/r06f_rk_$pw.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['nat_random_keys']
print(sys.argv[2], d['value'], d['ms_per_step'], d['kernel'], d['kernel_ms_per_launch'], d['parity']['match'])" $O/r06f_rk_$pw.json "random pipe=$pw"
done
done
