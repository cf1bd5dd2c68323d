#!/bin/bash
# what the per-launch timing events cost a step: VIGPATH_KTIME=1 (default) vs 0
set -o pipefail
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
T=r03y
for v in 1 0 1 0; do
  VIGPATH_KTIME=$v timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --no-extra --steps 40 > $O/${T}_k$v.log 2>&1 || exit $?
  grep '^{' $O/${T}_k$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ktime $v', d['ms_per_step'], d['roofline']['kernel_ms_per_launch'], d['parity']['match'])"
done
for v in 1 0; do
  VIGPATH_KTIME=$v timeout -k 10 400 python3 tools/bench_nf.py --only bridge,lb,fw,pol --no-cpu > $O/${T}_nf_k$v.log 2>&1 || exit $?
  grep '^{' $O/${T}_nf_k$v.log | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('ktime $v', d['value'])"
done
rm -rf $O/${T}_kt
VIGPATH_KTIME=0 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/${T}_kt -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu --no-e2e --no-extra > $O/${T}_kt.log 2>&1 || exit $?
