#!/bin/bash
# round 6 session g: the build after the round's kernel changes -- every GPU
# test, smoke, the default bench line, the headline's kernel trace and PMC
# passes (headline workload only), and the 2-rank gloo rehearsal of the N > 1
# line with its three modes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_session.sh r06g tests smoke bench trace pmc && BENCH_ARGS="--steps 5 --warmup 2" bash tools/gpu_session.sh r06g shard2
