#!/bin/bash
# round 5 session m (rerun as m2: lean-tile misses stay in their slices; the rewrite before the counters come back): expiry in one scan (the floor found beside the expired
# set), one read-back, one sort -- GPU tests (expiry-heavy ones included),
# churn rate and trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05m_pytest.out 2>&1 || { tail -40 gpurun_out/r05m_pytest.out; exit 1; }
tail -1 gpurun_out/r05m_pytest.out
timeout -k 10 300 python3 tools/bench_extra.py nat_churn > gpurun_out/r05m_churn.out 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*\|"match": [a-z]*\|"state_match": [a-z]*' gpurun_out/r05m_churn.out | tr '\n' ' '; echo
rm -rf gpurun_out/r05m_kt
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05m_kt -- python3 tools/bench_extra.py nat_churn > gpurun_out/r05m_kt.log 2>&1 || exit 1
