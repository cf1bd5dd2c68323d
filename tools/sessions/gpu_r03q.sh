#!/bin/bash
# N > 1 rehearsal on one GPU: 2 ranks sharing GPU 0 over gloo (both dictionary
# placements), and the owner pipeline's stage profile with every key routed
set -o pipefail
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
T=r03q
VIGPATH_COMM=host timeout -k 10 900 python3 bench.py --gpus 2 --no-cpu --no-e2e --steps 5 --warmup 2 > $O/${T}_shard2.log 2>&1 || exit $?
VIGPATH_PHASES=1 timeout -k 10 300 python3 bench.py --route-all --no-cpu --no-e2e --no-extra > $O/${T}_routeall.log 2>&1 || exit $?
