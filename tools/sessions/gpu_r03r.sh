#!/bin/bash
set -o pipefail
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
T=r03r
timeout -k 10 300 python3 bench.py --route-all --no-cpu --no-e2e --no-extra > $O/${T}_routeall.log 2>&1 || exit $?
rm -rf $O/${T}_kt
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/${T}_kt -- \
  python3 bench.py --route-all --no-cpu --no-e2e --no-extra --steps 4 --warmup 2 > $O/${T}_kt.log 2>&1 || exit $?
