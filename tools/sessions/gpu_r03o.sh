#!/bin/bash
# round-3 headline evidence: full GPU tests, smoke, bench, kernel trace,
# FETCH/WRITE PMC passes, wide-slot sweep, NF bench
set -o pipefail
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
T=r03o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/${T}_pytest.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py > $O/${T}_bench.log 2>&1 || exit $?
rm -rf $O/${T}_kt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_kt -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu --no-e2e > $O/${T}_kt.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf $O/${T}_$c
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/${T}_$c -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu --no-e2e --no-extra > $O/${T}_$c.log 2>&1 || exit $?
done
for sl in 128 256 512 1536; do
  timeout -k 10 300 python3 bench.py --slot $sl --no-cpu --no-e2e --no-extra >> $O/${T}_slots.log 2>&1 || exit $?
done
timeout -k 10 600 python3 tools/bench_nf.py --no-cpu > $O/${T}_nf.log 2>&1 || exit $?
