#!/bin/bash
# round 6 session am: the 64-byte tile kernel at two 512-thread blocks per CU
# (VIGPATH_TILE_WAVES=8, nat_classify64h) against one 1024-thread block
# (nat_classify64w): the bench-shape golden tests with it, then the headline
# interleaved twice (each line probes its kernel's own block shape)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
VIGPATH_TILE_WAVES=8 timeout -k 10 600 python -u -m pytest tests/test_golden.py tests/test_nat_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread \
  > $O/r06am_pytest.log 2>&1 || { tail -40 $O/r06am_pytest.log; exit 1; }
tail -1 $O/r06am_pytest.log
for i in 1 2; do
  for w in 16 8; do
    VIGPATH_TILE_WAVES=$w timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --no-extra > $O/r06am_rr_${w}_$i.json 2> $O/r06am_rr_${w}_$i.err || { tail -20 $O/r06am_rr_${w}_$i.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print('waves', sys.argv[2], d['value'], d['ms_per_step'], r.get('kernel'), r.get('kernel_ms_per_launch'), r.get('frac'), r.get('frac_step'), r.get('shape_ceiling_ms'), r.get('kernel_over_ceiling'), d['parity']['match'])" $O/r06am_rr_${w}_$i.json $w
  done
done
