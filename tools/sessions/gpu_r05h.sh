#!/bin/bash
# round 5 session h: new flows without sorting (tbl_new_keys_unsorted: phase A
# leaves each miss's key, a tagged key set gives first/last packets, first
# sightings ranked by a bit per position) -- GPU tests, then the churn
# workload against the sorted path (VIGPATH_NK_SORTED=1), interleaved
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05h_pytest.out 2>&1 || { tail -40 gpurun_out/r05h_pytest.out; exit 1; }
tail -1 gpurun_out/r05h_pytest.out
for i in 1 2; do
  for s in 1 0; do
    VIGPATH_NK_SORTED=$s timeout -k 10 300 python3 tools/bench_extra.py nat_churn > gpurun_out/r05h_churn_s${s}_$i.out 2>&1 || { tail -20 gpurun_out/r05h_churn_s${s}_$i.out; exit 1; }
    echo "sorted=$s $(grep -o '"ms_per_step": [0-9.]*\|"match": [a-z]*\|"state_match": [a-z]*' gpurun_out/r05h_churn_s${s}_$i.out | tr '\n' ' ')"
  done
done
