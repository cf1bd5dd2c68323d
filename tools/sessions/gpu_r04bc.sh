#!/bin/bash
# round 4 session bc: 128 touch bins, two run words per block and bin, two
# fold blocks per bin, against the previous commit (256 bins, one run word;
# abtmp/): GPU suite, then round robin, uniform order, viglb and vigbridge
# interleaved
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_session.sh r04bc tests || { tail -40 gpurun_out/r04bc_pytest.log; exit 1; }
grep -o "[0-9]* passed.*" gpurun_out/r04bc_pytest.log | tail -1
for v in old new old new old new; do
  d=.; [ $v = old ] && d=abtmp
  (cd $d && timeout -k 10 200 python3 bench.py --no-cpu --no-e2e --no-extra --steps 20) > gpurun_out/r04bc_r_$v.out 2>&1 || exit $?
  (cd $d && timeout -k 10 200 python3 bench.py --order uniform --no-cpu --no-e2e --no-extra --steps 20) > gpurun_out/r04bc_u_$v.out 2>&1 || exit $?
  (cd $d && timeout -k 10 200 python3 tools/bench_extra.py config4_lb) > gpurun_out/r04bc_lb_$v.out 2>&1 || exit $?
  (cd $d && timeout -k 10 200 python3 tools/bench_extra.py config3_bridge) > gpurun_out/r04bc_br_$v.out 2>&1 || exit $?
  echo "$v rr $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*' gpurun_out/r04bc_r_$v.out | tr '\n' ' ') | uni $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*' gpurun_out/r04bc_u_$v.out | tr '\n' ' ') | lb $(grep -o '"ms_per_step": [0-9.]*\|"match": [a-z]*' gpurun_out/r04bc_lb_$v.out | tr '\n' ' ') | br $(grep -o '"ms_per_step": [0-9.]*\|"match": [a-z]*' gpurun_out/r04bc_br_$v.out | tr '\n' ' ')"
done
