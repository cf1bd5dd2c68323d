#!/bin/bash
# round 4 session bf: run words generalized to one per fold block of a bin
# (4 at 64 bins): 64 bins (VIGPATH_BIN_BITS=6) and the default 128 against
# the previous commit (abtmp/): GPU suite (default and 64 bins), then round
# robin, uniform order and viglb interleaved. At 64 bins the uniform classify
# runs 0.709 ms (0.746 at 128) but its fold reads every entry four times: the
# step stays 0.808 ms; round robin and viglb unchanged. Not kept (128 bins,
# two run words stay)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_session.sh r04bf tests || { tail -40 gpurun_out/r04bf_pytest.log; exit 1; }
grep -o "[0-9]* passed.*" gpurun_out/r04bf_pytest.log | tail -1
VIGPATH_BIN_BITS=6 timeout -k 10 500 python -u -m pytest tests/test_nat_gpu.py tests/test_golden.py tests/test_lb_gpu.py tests/test_fw_gpu.py tests/test_shard_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04bf_pytest6.out 2>&1 || { tail -30 gpurun_out/r04bf_pytest6.out; exit 1; }
tail -1 gpurun_out/r04bf_pytest6.out
for v in old new new6 old new new6; do
  d=.; [ $v = old ] && d=abtmp
  bb=; [ $v = new6 ] && bb=6
  (cd $d && VIGPATH_BIN_BITS=$bb timeout -k 10 200 python3 bench.py --no-cpu --no-e2e --no-extra --steps 20) > gpurun_out/r04bf_r_$v.out 2>&1 || exit $?
  (cd $d && VIGPATH_BIN_BITS=$bb timeout -k 10 200 python3 bench.py --order uniform --no-cpu --no-e2e --no-extra --steps 20) > gpurun_out/r04bf_u_$v.out 2>&1 || exit $?
  (cd $d && VIGPATH_BIN_BITS=$bb timeout -k 10 200 python3 tools/bench_extra.py config4_lb) > gpurun_out/r04bf_lb_$v.out 2>&1 || exit $?
  echo "$v rr $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*' gpurun_out/r04bf_r_$v.out | tr '\n' ' ') | uni $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*' gpurun_out/r04bf_u_$v.out | tr '\n' ' ') | lb $(grep -o '"ms_per_step": [0-9.]*\|"match": [a-z]*' gpurun_out/r04bf_lb_$v.out | tr '\n' ' ')"
done
