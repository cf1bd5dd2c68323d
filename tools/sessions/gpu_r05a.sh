#!/bin/bash
# round 5 session a: baseline on this round's box -- route-all owner pipeline
# (stage times) and the default bench without the CPU leg
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --route-all --no-cpu --no-e2e --no-extra > gpurun_out/r05a_routeall.out 2>&1 || { tail -20 gpurun_out/r05a_routeall.out; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"stages_ms": {[^}]*}' gpurun_out/r05a_routeall.out
timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --no-extra > gpurun_out/r05a_bench.out 2>&1 || { tail -20 gpurun_out/r05a_bench.out; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*' gpurun_out/r05a_bench.out
