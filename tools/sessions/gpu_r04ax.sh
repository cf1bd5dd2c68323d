#!/bin/bash
# round 4 session ax: vignat's phase-B kernels (nat_miss_keys,
# nat_miss_finish) gather and store 64-byte slots four lanes per frame
# through LDS: vignat GPU tests, then the churn workload against the
# previous commit (abtmp/), interleaved, and a trace of the new one
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_nat_gpu.py tests/test_golden.py tests/test_mbuf_gpu.py tests/test_shard_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ax_pytest.out 2>&1 || { tail -30 gpurun_out/r04ax_pytest.out; exit 1; }
tail -1 gpurun_out/r04ax_pytest.out
for v in old new old new old new; do
  d=.; [ $v = old ] && d=abtmp
  (cd $d && timeout -k 10 200 python3 tools/bench_extra.py nat_churn) > gpurun_out/r04ax_ch_$v.out 2>&1 || exit $?
  echo "$v churn $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*\|"state_match": [a-z]*' gpurun_out/r04ax_ch_$v.out | tr '\n' ' ')"
done
rm -rf gpurun_out/r04ax_ch_kt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04ax_ch_kt -- python3 tools/bench_extra.py nat_churn > gpurun_out/r04ax_ch_kt.log 2>&1 || exit $?
