#!/bin/bash
# round 4 session bi: touch-bin entries stored through (sc1) instead of held
# in the L2 as partly written slice lines, against the previous commit
# (abtmp/): vignat/golden/lb tests, then round robin, uniform, viglb
# Uniform order slower (0.809 -> 0.839 ms per step, classify 0.747 ->
# 0.775): each 4-byte entry then goes out alone. Not kept
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_nat_gpu.py tests/test_golden.py tests/test_lb_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04bi_pytest.out 2>&1 || { tail -30 gpurun_out/r04bi_pytest.out; exit 1; }
tail -1 gpurun_out/r04bi_pytest.out
for v in old new old new old new; do
  d=.; [ $v = old ] && d=abtmp
  (cd $d && timeout -k 10 200 python3 bench.py --no-cpu --no-e2e --no-extra --steps 20) > gpurun_out/r04bi_r_$v.out 2>&1 || exit $?
  (cd $d && timeout -k 10 200 python3 bench.py --order uniform --no-cpu --no-e2e --no-extra --steps 20) > gpurun_out/r04bi_u_$v.out 2>&1 || exit $?
  (cd $d && timeout -k 10 200 python3 tools/bench_extra.py config4_lb) > gpurun_out/r04bi_lb_$v.out 2>&1 || exit $?
  echo "$v rr $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*' gpurun_out/r04bi_r_$v.out | tr '\n' ' ') | uni $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*' gpurun_out/r04bi_u_$v.out | tr '\n' ' ') | lb $(grep -o '"ms_per_step": [0-9.]*\|"match": [a-z]*' gpurun_out/r04bi_lb_$v.out | tr '\n' ' ')"
done
