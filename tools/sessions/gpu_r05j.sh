#!/bin/bash
# round 5 session j: kernel trace of the churn workload (unsorted new keys)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/r05j_kt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05j_kt -- python3 tools/bench_extra.py nat_churn > gpurun_out/r05j_kt.log 2>&1 || { tail -20 gpurun_out/r05j_kt.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05j_kt.log
