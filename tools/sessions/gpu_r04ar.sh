#!/bin/bash
# round 4 session ar: kernel trace of the uniform order (where the step
# spends its 54 us past the classify)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/r04ar_kt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04ar_kt -- python3 bench.py --order uniform --steps 10 --warmup 2 --no-cpu --no-e2e --no-extra > gpurun_out/r04ar_kt.log 2>&1 || exit $?
grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*' gpurun_out/r04ar_kt.log | tr '\n' ' '
