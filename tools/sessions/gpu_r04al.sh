#!/bin/bash
# round 4 session al: HBM traffic of the 128-byte-slot classify (FETCH_SIZE,
# WRITE_SIZE passes)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
BENCH_ARGS="--slot 128 --no-extra" bash tools/gpu_session.sh r04al pmc
