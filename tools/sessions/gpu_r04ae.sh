#!/bin/bash
# round 4 session ae: kernel trace of the random-key workload (two buckets
# per index, run words)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04ae_random_kt -- python3 tools/bench_extra.py nat_random_keys > gpurun_out/r04ae_random.out 2>&1 || exit $?
grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*' gpurun_out/r04ae_random.out
