#!/bin/bash
# final check of the committed build: GPU tests, smoke, default bench
set -o pipefail
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
T=r03zj
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/${T}_pytest.log 2>&1 || exit $?
tail -1 $O/${T}_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 || exit $?
tail -1 $O/${T}_smoke.log
timeout -k 10 400 python3 bench.py > $O/${T}_bench.log 2>&1 || exit $?
grep '^{' $O/${T}_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('bench', d['value'], d['ms_per_step'], r['kernel_ms_per_launch'], r['frac'], r['frac_step'], d['secondary_order']['value'], d['cpu_baseline']['value'], d['end_to_end']['value'], d['parity']['match'])"
