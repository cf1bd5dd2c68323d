#!/bin/bash
set -o pipefail
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
T=r03p
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "fw or bridge or spec or golden or shim" > $O/${T}_pytest.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/bench_nf.py --only bridge,fw --no-cpu > $O/${T}_nf.log 2>&1 || exit $?
for nf in pol lb fw; do
  for c in FETCH_SIZE WRITE_SIZE; do
    rm -rf $O/${T}_${nf}_$c
    PROF_KERNEL=${nf}_classify64 timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/${T}_${nf}_$c -- \
      python3 tools/bench_nf.py --only $nf --no-cpu --steps 3 > $O/${T}_${nf}_$c.log 2>&1 || exit $?
  done
done
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "wide or edge" > $O/${T}_pytest_wide0.log 2>&1 || exit $?
VIGPATH_W128_FULL=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "wide or edge" > $O/${T}_pytest_wide1.log 2>&1 || exit $?
for f in 0 1 0 1; do
  VIGPATH_W128_FULL=$f timeout -k 10 300 python3 bench.py --slot 128 --no-cpu --no-e2e --no-extra >> $O/${T}_w128_$f.log 2>&1 || exit $?
done
