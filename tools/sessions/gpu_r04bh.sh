#!/bin/bash
# round 4 session bh: the uniform order's counters (FETCH_SIZE, WRITE_SIZE,
# TCC hit/miss passes) and kernel trace at 128 touch bins
cd "${GRAFT_REPO_ROOT:-/root/repo}"
BENCH_ARGS="--order uniform --no-extra" bash tools/gpu_session.sh r04bh_uni trace pmc || exit $?
bash tools/pmc_tcc.sh r04bh_uni --order uniform || exit $?
bash tools/pmc_tcc.sh r04bh_rr || exit $?
echo done
