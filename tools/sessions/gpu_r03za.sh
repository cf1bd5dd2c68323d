#!/bin/bash
# host API trace beside the kernel trace without timing events; owner route-all step
set -o pipefail
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
T=r03za
rm -rf $O/${T}_ht
timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/${T}_ht -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu --no-e2e --no-extra > $O/${T}_ht.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --route-all --no-cpu --no-e2e --no-extra --steps 20 > $O/${T}_ra.log 2>&1 || exit $?
grep '^{' $O/${T}_ra.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('route-all', d['value'], d['ms_per_step'], d['parity'])"
