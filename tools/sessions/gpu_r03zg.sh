#!/bin/bash
# route_pad folded into route_scan; timing-switch test: GPU tests + route-all
set -o pipefail
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
T=r03zg
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/${T}_pytest.log 2>&1 || exit $?
tail -1 $O/${T}_pytest.log
for i in 1 2; do
timeout -k 10 400 python3 bench.py --route-all --no-cpu --no-e2e --no-extra --steps 20 > $O/${T}_ra$i.log 2>&1 || exit $?
grep '^{' $O/${T}_ra$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('route-all', d['value'], d['ms_per_step'], d['parity']['match'])"
done
