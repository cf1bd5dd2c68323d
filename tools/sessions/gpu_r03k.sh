#!/bin/bash
# round-3 diagnostics: bridge write traffic on a re-used batch, the uniform-row
# probe ceiling, kernel traces of vigpol / viglb steps and of the headline bench
set -o pipefail
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
T=r03k
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/${T}_pytest.log 2>&1 || exit $?
for u in 8 16 32; do
  VIGPATH_FOLD_U=$u timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --no-extra > $O/${T}_fold$u.log 2>&1 || exit $?
done
for c in WRITE_SIZE FETCH_SIZE; do
  rm -rf $O/${T}_brsame_$c
  BENCH_NF_SAME=1 timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/${T}_brsame_$c -- \
    python3 tools/bench_nf.py --only bridge --no-cpu --steps 3 > $O/${T}_brsame_$c.log 2>&1 || exit $?
done
timeout -k 10 300 tools/stream_probe r > $O/${T}_probe_rand.log 2>&1 || exit $?
rm -rf $O/${T}_nfkt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_nfkt -- \
  python3 tools/bench_nf.py --only pol,lb --no-cpu --steps 3 > $O/${T}_nfkt.log 2>&1 || exit $?
rm -rf $O/${T}_kt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_kt -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu --no-e2e > $O/${T}_kt.log 2>&1 || exit $?
