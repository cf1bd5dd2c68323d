#!/bin/bash
# round 6 session b: the 1024-thread vignat tile with its block range cut into
# 2 or 4 contiguous sub-ranges (VIGPATH_SPLIT: the streams of 256-thread
# blocks, one table copy per CU) -- vignat tests at split 4, then an A/B of
# split 1/2/4 and the 256-thread kernel in round robin and uniform order,
# each with its own shape ceiling
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
VIGPATH_SPLIT=4 timeout -k 10 600 python -u -m pytest tests/test_nat_gpu.py tests/test_golden.py \
  tests/test_layout_gpu.py -x -q --timeout 200 --timeout-method thread \
  > $O/r06b_split4.log 2>&1 || { tail -30 $O/r06b_split4.log; exit 1; }
tail -1 $O/r06b_split4.log
for i in 1 2; do
for order in rr uniform; do
for v in s1 s2 s4 w4; do
  case $v in s*) env="VIGPATH_SPLIT=${v#s}";; w4) env="VIGPATH_BLOCK_WAVES=4";; esac
  env $env timeout -k 10 300 python3 bench.py --order $order --no-cpu --no-e2e --no-extra --steps 10 \
    > $O/r06b_ab_${order}_$v.json 2> $O/r06b_ab_${order}_$v.err || { tail -20 $O/r06b_ab_${order}_$v.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print(sys.argv[2], d['value'], d['ms_per_step'], r['kernel'], r['kernel_ms_per_launch'], r.get('shape_ceiling_ms'), r.get('kernel_over_ceiling'))" $O/r06b_ab_${order}_$v.json "$order $v"
done
done
done
