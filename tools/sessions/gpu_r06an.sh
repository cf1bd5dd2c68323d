#!/bin/bash
# round 6 session an: the 64-byte tile kernel by block shape with the owner
# paths compiled out -- 16 (nat_classify64w), 8 (nat_classify64h), 4
# (nat_classify64q) waves per block: the golden tests with 4, then the
# headline interleaved twice (each line probes its kernel's own shape)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
VIGPATH_TILE_WAVES=4 timeout -k 10 600 python -u -m pytest tests/test_golden.py tests/test_nat_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread \
  > $O/r06an_pytest.log 2>&1 || { tail -40 $O/r06an_pytest.log; exit 1; }
tail -1 $O/r06an_pytest.log
for i in 1 2; do
  for w in 16 8 4; do
    VIGPATH_TILE_WAVES=$w timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --no-extra > $O/r06an_rr_${w}_$i.json 2> $O/r06an_rr_${w}_$i.err || { tail -20 $O/r06an_rr_${w}_$i.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print('waves', sys.argv[2], d['value'], d['ms_per_step'], r.get('kernel'), r.get('kernel_ms_per_launch'), r.get('frac'), r.get('frac_step'), r.get('shape_ceiling_ms'), r.get('kernel_over_ceiling'), d['parity']['match'])" $O/r06an_rr_${w}_$i.json $w
  done
done
