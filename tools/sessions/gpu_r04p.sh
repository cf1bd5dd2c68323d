#!/bin/bash
# round 4 session p: register-path phase-B kernels (nat_miss_keys /
# nat_miss_finish): GPU suite, churn, headline, churn trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_session.sh r04p tests || exit $?
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/bench_extra.py nat_churn > gpurun_out/r04p_churn.out 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --no-cpu --no-e2e --no-extra --steps 10 > gpurun_out/r04p_head.out 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04p_churn_kt -- python3 tools/bench_extra.py nat_churn > gpurun_out/r04p_churn_kt.log 2>&1 || exit $?
grep -o '"value": [0-9.]*, "unit": "Mpps", "ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*\|"state_match": [a-z]*' gpurun_out/r04p_churn.out gpurun_out/r04p_head.out
