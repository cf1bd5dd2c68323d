#!/bin/bash
# round 4 session bd: vigbridge back at 256 bins (two run words kept) against
# the previous commit (abtmp/): bridge GPU tests, config3_bridge interleaved
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_bridge_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04bd_pytest.out 2>&1 || { tail -30 gpurun_out/r04bd_pytest.out; exit 1; }
tail -1 gpurun_out/r04bd_pytest.out
for v in old new old new old new; do
  d=.; [ $v = old ] && d=abtmp
  (cd $d && timeout -k 10 200 python3 tools/bench_extra.py config3_bridge) > gpurun_out/r04bd_br_$v.out 2>&1 || exit $?
  echo "$v br $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*' gpurun_out/r04bd_br_$v.out | tr '\n' ' ')"
done
