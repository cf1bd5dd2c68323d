#!/bin/bash
# vigpol / viglb rework: tests, NF bench, kernel trace; bridge write traffic on a re-used batch
set -o pipefail
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
T=r03l
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "pol or lb or spec or golden or shim" > $O/${T}_pytest.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/bench_nf.py --only pol,lb --no-cpu > $O/${T}_nf.log 2>&1 || exit $?
rm -rf $O/${T}_nfkt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_nfkt -- \
  python3 tools/bench_nf.py --only pol,lb --no-cpu --steps 3 > $O/${T}_nfkt.log 2>&1 || exit $?
for c in WRITE_SIZE FETCH_SIZE; do
  rm -rf $O/${T}_brsame_$c
  BENCH_NF_SAME=1 timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/${T}_brsame_$c -- \
    python3 tools/bench_nf.py --only bridge --no-cpu --steps 3 > $O/${T}_brsame_$c.log 2>&1 || exit $?
done
