#!/bin/bash
# round 6 session a: GPU tests, smoke and the default bench line of the tree
# as round 5 left it plus the ABI/bench changes; the pipelined vignat tiles
# (VIGPATH_PIPE=8 / 12) through the vignat tests, then an A/B against the
# default 1024-thread tiles in round robin and uniform order
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
bash tools/gpu_session.sh r06a tests smoke bench || exit $?
for pw in 8 12; do
  VIGPATH_PIPE=$pw timeout -k 10 600 python -u -m pytest tests/test_nat_gpu.py tests/test_golden.py \
    tests/test_layout_gpu.py tests/test_spec_gpu.py -x -q --timeout 200 --timeout-method thread \
    > $O/r06a_pipe$pw.log 2>&1 || { tail -30 $O/r06a_pipe$pw.log; exit 1; }
  tail -1 $O/r06a_pipe$pw.log
done
for i in 1 2; do
for order in rr uniform; do
for pw in 0 8 12; do
  VIGPATH_PIPE=$pw timeout -k 10 300 python3 bench.py --order $order --no-cpu --no-e2e --no-extra --steps 10 \
    > $O/r06a_ab_${order}_$pw.json 2> $O/r06a_ab_${order}_$pw.err || { tail -20 $O/r06a_ab_${order}_$pw.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print(sys.argv[2], d['value'], d['ms_per_step'], r['kernel'], r['kernel_ms_per_launch'], r.get('kernel_over_ceiling'))" $O/r06a_ab_${order}_$pw.json "$order pipe=$pw"
done
done
done
