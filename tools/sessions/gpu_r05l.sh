#!/bin/bash
# round 5 session l: is the headline classify slower with phase A's miss-key
# writes (compiled in, idle in steady state)? And the churn classify with the
# sorted path (no key writes at run time), traced
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
timeout -k 10 200 python3 bench.py --no-cpu --no-e2e --no-extra > gpurun_out/r05l_bench_$i.out 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*' gpurun_out/r05l_bench_$i.out | head -2 | tr '\n' ' '; echo
done
rm -rf gpurun_out/r05l_kt
VIGPATH_NK_SORTED=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05l_kt -- python3 tools/bench_extra.py nat_churn > gpurun_out/r05l_kt.log 2>&1 || exit 1
