#!/bin/bash
# round-3 measurement session (tests, bench, NF bench, bridge write-traffic PMC)
set -o pipefail
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
T=r03j
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/${T}_pytest.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py > $O/${T}_bench.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/bench_nf.py --no-cpu > $O/${T}_nf.log 2>&1 || exit $?
for bins in 1 0; do
  rm -rf $O/${T}_brw_b$bins
  VIGPATH_TOUCH_BINS=$bins timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${T}_brw_b$bins -- \
    python3 tools/bench_nf.py --only bridge --no-cpu --steps 3 > $O/${T}_brw_b$bins.log 2>&1 || exit $?
done
