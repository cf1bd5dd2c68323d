#!/bin/bash
# owner route-all pipeline: kernel + HIP API trace (no timing events)
set -o pipefail
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
T=r03zc
rm -rf $O/${T}_ht
timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace --output-format csv -d $O/${T}_ht -- \
  python3 bench.py --route-all --steps 6 --warmup 2 --no-cpu --no-e2e --no-extra > $O/${T}_ht.log 2>&1 || exit $?
