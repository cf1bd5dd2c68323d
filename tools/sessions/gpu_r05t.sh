#!/bin/bash
# round 5 session t: viglb / vigfw flow hashes with batched LDS reads
# (crc13_lds) -- their GPU tests, then the full bench line (config4_lb)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_lb_gpu.py tests/test_fw_gpu.py tests/test_nf_shim_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05t_pytest.out 2>&1 || { tail -40 gpurun_out/r05t_pytest.out; exit 1; }
tail -1 gpurun_out/r05t_pytest.out
timeout -k 10 600 python3 bench.py > gpurun_out/r05t_bench.json 2> gpurun_out/r05t_bench.err || { tail -20 gpurun_out/r05t_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r05t_bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'])
for k in ('config4_lb','config3_bridge','nat_random_keys','nat_churn','secondary_order'):
  e=d.get(k) or {}
  print(k, {x: e.get(x) for x in ('value','ms_per_step','kernel_ms_per_launch','frac','match')})"
