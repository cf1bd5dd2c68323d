#!/bin/bash
# round 4 session bb: 128 touch bins with two fold blocks per bin (the fold
# keeps 256 blocks) against the previous commit's 256 bins (abtmp/), and
# 64 bins x 4 (VIGPATH_BIN_BITS=6): GPU suite, then round robin, uniform
# order and viglb interleaved. Classify faster with fewer bins (uniform 0.786
# -> 0.747 / 0.711 ms) but the step slower: a block has one run word per
# bin, so at 128 bins half of its runs fall back to entries (rr step 0.474
# -> 0.488 / 0.520 ms). Not kept
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_session.sh r04bb tests || { tail -40 gpurun_out/r04bb_pytest.log; exit 1; }
grep -o "[0-9]* passed.*" gpurun_out/r04bb_pytest.log | tail -1
for v in old new new6 old new new6; do
  d=.; [ $v = old ] && d=abtmp
  bb=; [ $v = new6 ] && bb=6
  (cd $d && VIGPATH_BIN_BITS=$bb timeout -k 10 200 python3 bench.py --no-cpu --no-e2e --no-extra --steps 20) > gpurun_out/r04bb_r_$v.out 2>&1 || exit $?
  (cd $d && VIGPATH_BIN_BITS=$bb timeout -k 10 200 python3 bench.py --order uniform --no-cpu --no-e2e --no-extra --steps 20) > gpurun_out/r04bb_u_$v.out 2>&1 || exit $?
  (cd $d && VIGPATH_BIN_BITS=$bb timeout -k 10 200 python3 tools/bench_extra.py config4_lb) > gpurun_out/r04bb_lb_$v.out 2>&1 || exit $?
  echo "$v rr $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*' gpurun_out/r04bb_r_$v.out | tr '\n' ' ') | uni $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*' gpurun_out/r04bb_u_$v.out | tr '\n' ' ') | lb $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*' gpurun_out/r04bb_lb_$v.out | tr '\n' ' ')"
done
