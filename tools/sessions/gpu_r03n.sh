#!/bin/bash
# bridge without scratch arrays: tests, NF bench, PMC write/fetch; vigpol register runs
set -o pipefail
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
T=r03n
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "bridge or pol or spec or golden or shim" > $O/${T}_pytest.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/bench_nf.py --only bridge,flood,pol --no-cpu > $O/${T}_nf.log 2>&1 || exit $?
for c in WRITE_SIZE FETCH_SIZE; do
  rm -rf $O/${T}_br_$c
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/${T}_br_$c -- \
    python3 tools/bench_nf.py --only bridge --no-cpu --steps 3 > $O/${T}_br_$c.log 2>&1 || exit $?
done
