#!/bin/bash
# round 4 session aa: the fold with run words loaded beside the counts:
# GPU suite (touch-bin users), kernel trace of the headline, bench defaults
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_session.sh r04aa tests || exit $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04aa_kt -- python3 bench.py --no-cpu --no-e2e --no-extra --steps 20 > gpurun_out/r04aa_kt.log 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --no-cpu --no-e2e --no-extra --steps 20 > gpurun_out/r04aa_head.out 2>&1 || exit $?
grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*' gpurun_out/r04aa_head.out
