#!/bin/bash
# owner-mode lean pass 1: tests, route-all profile, 2-rank rehearsal
set -o pipefail
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
T=r03t
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "nat or shard or owner or golden or spec or layout" > $O/${T}_pytest.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --route-all --no-cpu --no-e2e --no-extra > $O/${T}_routeall.log 2>&1 || exit $?
VIGPATH_PHASES=1 timeout -k 10 300 python3 bench.py --route-all --no-cpu --no-e2e --no-extra --steps 4 > $O/${T}_routeall_phases.log 2>&1 || exit $?
VIGPATH_COMM=host timeout -k 10 900 python3 bench.py --gpus 2 --no-cpu --no-e2e --no-extra --steps 3 --warmup 2 > $O/${T}_shard2.log 2>&1 || exit $?
