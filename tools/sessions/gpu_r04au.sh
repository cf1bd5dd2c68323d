#!/bin/bash
# round 4 session au: kernel traces of the random-key and churn workloads
# (where their steps spend the time past the classify)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in nat_random_keys nat_churn config4_lb; do
  rm -rf gpurun_out/r04au_$w
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04au_$w -- python3 tools/bench_extra.py $w > gpurun_out/r04au_$w.log 2>&1 || exit $?
  grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*' gpurun_out/r04au_$w.log | tr '\n' ' '; echo
done
