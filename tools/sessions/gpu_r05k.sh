#!/bin/bash
# round 5 session k: churn with filtered key-set atomics; trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_nat_gpu.py tests/test_golden.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05k_pytest.out 2>&1 || { tail -30 gpurun_out/r05k_pytest.out; exit 1; }
tail -1 gpurun_out/r05k_pytest.out
timeout -k 10 300 python3 tools/bench_extra.py nat_churn > gpurun_out/r05k_churn.out 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*\|"match": [a-z]*\|"state_match": [a-z]*' gpurun_out/r05k_churn.out | tr '\n' ' '; echo
rm -rf gpurun_out/r05k_kt
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05k_kt -- python3 tools/bench_extra.py nat_churn > gpurun_out/r05k_kt.log 2>&1 || exit 1
