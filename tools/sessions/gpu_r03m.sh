#!/bin/bash
set -o pipefail
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
T=r03m
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/${T}_pytest.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/bench_nf.py --no-cpu > $O/${T}_nf.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py > $O/${T}_bench.log 2>&1 || exit $?
