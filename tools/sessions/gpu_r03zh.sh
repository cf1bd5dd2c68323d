#!/bin/bash
# fold reads each wave's slices as one dense entry list: GPU tests, bench,
# NF bench, kernel trace (fold duration)
set -o pipefail
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
T=r03zh
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/${T}_pytest.log 2>&1 || exit $?
tail -1 $O/${T}_pytest.log
timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --no-extra --steps 40 > $O/${T}_b40.log 2>&1 || exit $?
grep '^{' $O/${T}_b40.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('bench40', d['value'], d['ms_per_step'], r['kernel_ms_per_launch'], r['frac_step'], d['parity']['match'])"
timeout -k 10 600 python3 tools/bench_nf.py --no-cpu > $O/${T}_nf.log 2>&1 || exit $?
grep '^{' $O/${T}_nf.log | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print(d['workload'][:30], d['value'], d['kernel_mpps'])"
rm -rf $O/${T}_kt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_kt -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu --no-e2e --no-extra > $O/${T}_kt.log 2>&1 || exit $?
rm -rf $O/${T}_nfkt
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/${T}_nfkt -- \
  python3 tools/bench_nf.py --only bridge,fw --no-cpu --steps 4 > $O/${T}_nfkt.log 2>&1 || exit $?
