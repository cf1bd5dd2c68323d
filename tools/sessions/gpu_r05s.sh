#!/bin/bash
# round 5 session s: one port per burst (vp_dev_batch.in_port) -- the GPU
# suite, then bench A/B: the burst's port vs a per-packet port array, twice
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05s_pytest.out 2>&1 || { tail -40 gpurun_out/r05s_pytest.out; exit 1; }
tail -1 gpurun_out/r05s_pytest.out
for i in 1 2; do
for v in "" "--port-array"; do
timeout -k 10 300 python3 bench.py --no-extra --no-cpu --no-e2e $v > gpurun_out/r05s_b$i$v.json 2> gpurun_out/r05s_b$i$v.err || { tail -20 gpurun_out/r05s_b$i$v.err; exit 1; }
python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2] or 'burst', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'], d['roofline']['frac'])" gpurun_out/r05s_b$i$v.json "$v"
done
done
