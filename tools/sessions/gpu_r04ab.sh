#!/bin/bash
# round 4 session ab: 16M flows on one GPU (config 5's per-GPU table), and
# the uniform packet order, after this round's table and fold changes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --flows 16777216 --no-cpu --no-e2e --no-extra --steps 10 > gpurun_out/r04ab_16m.out 2>&1 || exit $?
grep -o '"value": [0-9.]*, "unit": "Mpps", "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*' gpurun_out/r04ab_16m.out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04ab_16m_kt -- python3 bench.py --flows 16777216 --no-cpu --no-e2e --no-extra --steps 10 > gpurun_out/r04ab_16m_kt.log 2>&1 || exit $?
