#!/bin/bash
# round 4 session aj: frames64_tiles (viglb, vigfw, vigpol, vignat owner pass
# 2) issues at a raised wave priority: their GPU tests, then config4_lb
# against the previous commit's build in abtmp/, interleaved on one box
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_lb_gpu.py tests/test_fw_gpu.py tests/test_pol_gpu.py tests/test_shard_gpu.py tests/test_nf_shim_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04aj_pytest.out 2>&1 || { tail -30 gpurun_out/r04aj_pytest.out; exit 1; }
tail -1 gpurun_out/r04aj_pytest.out
for v in old new old new old new; do
  d=.; [ $v = old ] && d=abtmp
  timeout -k 10 200 python3 $d/tools/bench_extra.py config4_lb > gpurun_out/r04aj_$v.out 2>&1 || exit $?
  echo "$v $(grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*' gpurun_out/r04aj_$v.out | tr '\n' ' ')"
done
