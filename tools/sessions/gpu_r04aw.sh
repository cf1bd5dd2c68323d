#!/bin/bash
# round 4 session aw: the lean tile walks a full home bucket's probe path on
# in the lane (bounded, wave-uniform loop) instead of one extra bucket; the
# reprobe queue only for lanes past the bound: vignat GPU tests, then the
# headline
# and the random-key workload against the previous commit (abtmp/)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_nat_gpu.py tests/test_golden.py tests/test_mbuf_gpu.py tests/test_shard_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04aw_pytest.out 2>&1 || { tail -30 gpurun_out/r04aw_pytest.out; exit 1; }
tail -1 gpurun_out/r04aw_pytest.out
for v in old new old new old new; do
  d=.; [ $v = old ] && d=abtmp
  (cd $d && timeout -k 10 200 python3 bench.py --no-cpu --no-e2e --no-extra --steps 20) > gpurun_out/r04aw_$v.out 2>&1 || exit $?
  (cd $d && timeout -k 10 200 python3 tools/bench_extra.py nat_random_keys) > gpurun_out/r04aw_rk_$v.out 2>&1 || exit $?
  echo "$v $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*' gpurun_out/r04aw_$v.out | tr '\n' ' ') | rk $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*' gpurun_out/r04aw_rk_$v.out | tr '\n' ' ')"
done
rm -rf gpurun_out/r04aw_rk_kt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04aw_rk_kt -- python3 tools/bench_extra.py nat_random_keys > gpurun_out/r04aw_rk_kt.log 2>&1 || exit $?
