#!/bin/bash
# round 6 session ap: the final tree's side numbers -- every NF
# (tools/bench_nf.py), wide slots, the end-to-end host paths
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_session.sh r06ap nf slots:128,256,512,1536 e2e
