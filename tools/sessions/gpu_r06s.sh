#!/bin/bash
# round 6 session s: phase A's control block published by the classify's
# last block (tile_publish) -- the vignat tests, then the headline with it on
# and off (VIGPATH_TILE_PUB), interleaved, and the churn workload
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_nat_gpu.py tests/test_golden.py tests/test_layout_gpu.py tests/test_spec_gpu.py tests/test_mbuf_gpu.py -x -q \
  --timeout 200 --timeout-method thread > $O/r06s_pytest.log 2>&1 || { tail -40 $O/r06s_pytest.log; exit 1; }
tail -1 $O/r06s_pytest.log
for i in 1 2; do
  for p in 1 0; do
    VIGPATH_TILE_PUB=$p timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --no-extra > $O/r06s_rr_${p}_$i.json 2> $O/r06s_rr_${p}_$i.err || { tail -20 $O/r06s_rr_${p}_$i.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print('pub', sys.argv[2], d['value'], d['ms_per_step'], r.get('kernel_ms_per_launch'), r.get('frac'), r.get('frac_step'), d.get('new_flow_mpps'), d['parity']['match'])" $O/r06s_rr_${p}_$i.json $p
  done
done
VIGPATH_TILE_PUB=1 timeout -k 10 300 python3 tools/bench_extra.py nat_churn > $O/r06s_churn.json 2> $O/r06s_churn.err || { tail -20 $O/r06s_churn.err; exit 1; }
python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['nat_churn']
print('churn', d['value'], d['ms_per_step'], d['kernel'], d['kernel_ms_per_launch'], d['parity']['match'], d['parity'].get('state_match'))" $O/r06s_churn.json
