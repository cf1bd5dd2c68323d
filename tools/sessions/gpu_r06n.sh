#!/bin/bash
# round 6 session n: the build with the first-sighting cut and the preload --
# every GPU test, smoke, the default bench line, the headline's trace and PMC
# passes, and uniform order's PMC passes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_session.sh r06n tests smoke bench trace pmc && BENCH_ARGS="--order uniform" bash tools/gpu_session.sh r06nu pmc
