#!/bin/bash
# round 4 session bj: the lean tile's probe walk moved into a helper
# (lean_walk; same code): vignat, golden, mbuf and shard GPU tests, smoke,
# the headline and the random-key workload
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_nat_gpu.py tests/test_golden.py tests/test_mbuf_gpu.py tests/test_shard_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04bj_pytest.out 2>&1 || { tail -30 gpurun_out/r04bj_pytest.out; exit 1; }
tail -1 gpurun_out/r04bj_pytest.out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04bj_smoke.log 2>&1 || { tail -20 gpurun_out/r04bj_smoke.log; exit 1; }
tail -1 gpurun_out/r04bj_smoke.log
timeout -k 10 200 python3 bench.py --no-cpu --no-e2e --no-extra --steps 20 > gpurun_out/r04bj_r.out 2>&1 || exit $?
timeout -k 10 200 python3 tools/bench_extra.py nat_random_keys > gpurun_out/r04bj_rk.out 2>&1 || exit $?
echo "rr $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*' gpurun_out/r04bj_r.out | tr '\n' ' ') | rk $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*' gpurun_out/r04bj_rk.out | tr '\n' ' ')"
