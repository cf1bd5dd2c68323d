#!/bin/bash
# round 6 session a: the tree as round 5 left it plus the ABI/bench changes --
# GPU tests, smoke, the default bench line, and a 2-rank gloo rehearsal of the
# N > 1 line (owner, chunked owner, replicated)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_session.sh r06a tests smoke bench && BENCH_ARGS="--steps 5 --warmup 2" bash tools/gpu_session.sh r06a shard2
