#!/bin/bash
# round 4 session q: block-level atomics in tbl_min_ts / exp_collect / exp_apply,
# nk_dedup without redundant atomicMin: GPU suite, churn, headline, trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_session.sh r04q tests || exit $?
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/bench_extra.py nat_churn > gpurun_out/r04q_churn.out 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --no-cpu --no-e2e --no-extra --steps 10 > gpurun_out/r04q_head.out 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04q_churn_kt -- python3 tools/bench_extra.py nat_churn > gpurun_out/r04q_churn_kt.log 2>&1 || exit $?
grep -o '"value": [0-9.]*, "unit": "Mpps", "ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*\|"state_match": [a-z]*' gpurun_out/r04q_churn.out gpurun_out/r04q_head.out
