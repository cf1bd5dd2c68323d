#!/bin/bash
# round 6 session l: device code preloaded at context creation -- smoke, the
# vignat tests, and the first batch's host timeline and new-flow rate
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r06l_smoke.log 2>&1 || { tail -20 $O/r06l_smoke.log; exit 1; }
tail -1 $O/r06l_smoke.log
timeout -k 10 600 python -u -m pytest tests/test_nat_gpu.py -x -q --timeout 200 --timeout-method thread > $O/r06l_pytest.log 2>&1 || { tail -30 $O/r06l_pytest.log; exit 1; }
tail -1 $O/r06l_pytest.log
for i in 1 2; do
VIGPATH_HOSTPROF=1 timeout -k 10 300 python3 bench.py --steps 2 --warmup 2 --no-cpu --no-e2e --no-extra > $O/r06l_hp$i.json 2> $O/r06l_hp$i.err || { tail -20 $O/r06l_hp$i.err; exit 1; }
grep hostprof $O/r06l_hp$i.err | head -2
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('new_flow_mpps', d['new_flow_mpps'], 'value', d['value'])" $O/r06l_hp$i.json
done
