#!/bin/bash
# L2 (TCC) hit/miss counters of one bench configuration, one --pmc pass
# (tests and tools only; no product code): bash tools/pmc_tcc.sh TAG [bench args]
set -o pipefail
TAG=$1; shift
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
rm -rf $O/${TAG}_tcc
timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv \
  -d $O/${TAG}_tcc -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-e2e --no-extra "$@" \
  > $O/${TAG}_tcc.log 2>&1
