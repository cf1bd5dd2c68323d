#!/bin/bash
# round 4 session av: the lean tile probes a full home bucket's successor
# itself (one more round trip for the lanes that need it) instead of
# queueing the packet for nat_reprobe: vignat GPU tests, then the headline
# and the random-key workload against the previous commit (abtmp/)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_nat_gpu.py tests/test_golden.py tests/test_mbuf_gpu.py tests/test_shard_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04av_pytest.out 2>&1 || { tail -30 gpurun_out/r04av_pytest.out; exit 1; }
tail -1 gpurun_out/r04av_pytest.out
for v in old new old new old new; do
  d=.; [ $v = old ] && d=abtmp
  (cd $d && timeout -k 10 200 python3 bench.py --no-cpu --no-e2e --no-extra --steps 20) > gpurun_out/r04av_$v.out 2>&1 || exit $?
  (cd $d && timeout -k 10 200 python3 tools/bench_extra.py nat_random_keys) > gpurun_out/r04av_rk_$v.out 2>&1 || exit $?
  echo "$v $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*' gpurun_out/r04av_$v.out | tr '\n' ' ') | rk $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*' gpurun_out/r04av_rk_$v.out | tr '\n' ' ')"
done
