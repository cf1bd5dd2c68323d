#!/bin/bash
# round 4 session y: the owner pipeline after the sliced exchange and run
# words (--route-all on one GPU), and the 2-rank rehearsal of bench.py
# --gpus 2 (two ranks sharing GPU 0 over the host transport)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --route-all --no-cpu --no-e2e --no-extra --steps 10 > gpurun_out/r04y_routeall.out 2>&1 || exit $?
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"stages_ms": {[^}]*}}' gpurun_out/r04y_routeall.out
bash tools/gpu_session.sh r04y shard2 || exit $?
grep '^{' gpurun_out/r04y_shard2.log | head -c 3000
