#!/bin/bash
# round-3 close: 2-rank rehearsal of bench.py --gpus 2 (ranks share GPU 0
# over gloo), smoke, default bench, kernel trace of the default bench
set -o pipefail
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
T=r03ze
VIGPATH_COMM=host timeout -k 10 900 python3 bench.py --gpus 2 --no-cpu --no-e2e --steps 3 --warmup 2 > $O/${T}_shard2.log 2>&1 || exit $?
grep '^{' $O/${T}_shard2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('shard2', d['value'], d['ms_per_step'], d['config']['parallelism'], d['roofline']['kernel_ms_per_launch'], d.get('other_shard_mode'))"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py > $O/${T}_bench.log 2>&1 || exit $?
grep '^{' $O/${T}_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('bench', d['value'], d['ms_per_step'], r['kernel_ms_per_launch'], r['frac'], r['frac_step'], d['secondary_order']['value'], d['cpu_baseline']['value'], d['end_to_end']['value'], d['parity']['match'])"
rm -rf $O/${T}_kt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_kt -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu --no-e2e > $O/${T}_kt.log 2>&1 || exit $?
