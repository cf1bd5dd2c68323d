#!/bin/bash
# whole-slot stores in viglb, vigfw and owner pass 2
set -o pipefail
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
T=r03s
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "lb or fw or shard or owner or spec or golden or shim" > $O/${T}_pytest.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/bench_nf.py --only lb,fw --no-cpu > $O/${T}_nf.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --route-all --no-cpu --no-e2e --no-extra > $O/${T}_routeall.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "wide or edge" > $O/${T}_pytest_wide.log 2>&1 || exit $?
for sl in 128 256 1536; do
  timeout -k 10 300 python3 bench.py --slot $sl --no-cpu --no-e2e --no-extra >> $O/${T}_slots.log 2>&1 || exit $?
done
