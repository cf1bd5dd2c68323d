#!/bin/bash
# host vs device timeline of the steady-state step: kernel trace + HIP runtime API trace
set -o pipefail
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
T=r03x
rm -rf $O/${T}_ht
timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/${T}_ht -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu --no-e2e --no-extra > $O/${T}_ht.log 2>&1 || exit $?
VIGPATH_HOSTPROF=1 timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-e2e --no-extra > $O/${T}_hp.log 2>&1 || exit $?
