#!/bin/bash
# fold sweep: touch-bin count floor 2^8..2^10 (VIGPATH_BIN_BITS), step vs kernel
set -o pipefail
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
T=r03v
for bb in 8 9 10 8; do
  VIGPATH_BIN_BITS=$bb timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --no-extra --steps 40 > $O/${T}_bb$bb.log 2>&1 || exit $?
  grep '^{' $O/${T}_bb$bb.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bb', $bb, d['ms_per_step'], d['roofline']['kernel_ms_per_launch'], d['parity']['match'])"
done
rm -rf $O/${T}_kt
VIGPATH_BIN_BITS=9 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_kt -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu --no-e2e --no-extra > $O/${T}_kt.log 2>&1 || exit $?
rm -rf $O/${T}_nfkt
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/${T}_nfkt -- \
  python3 tools/bench_nf.py --only lb,fw,bridge,pol --no-cpu --steps 8 > $O/${T}_nfkt.log 2>&1 || exit $?
