#!/bin/bash
# headline without per-launch timing events (kernel time from a second pass):
# GPU tests, smoke, bench x2, NF bench, kernel trace of the headline pass
set -o pipefail
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
T=r03z
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/${T}_pytest.log 2>&1 || exit $?
tail -1 $O/${T}_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py > $O/${T}_bench.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --steps 40 > $O/${T}_bench40.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/bench_nf.py --no-cpu > $O/${T}_nf.log 2>&1 || exit $?
rm -rf $O/${T}_kt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_kt -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu --no-e2e > $O/${T}_kt.log 2>&1 || exit $?
