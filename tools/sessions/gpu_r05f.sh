#!/bin/bash
# round 5 session f: the whole GPU suite, smoke, and the default bench (with
# the shape ceiling and the per-packet drop-in rate)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05f_pytest.out 2>&1 || { tail -40 gpurun_out/r05f_pytest.out; exit 1; }
tail -1 gpurun_out/r05f_pytest.out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05f_smoke.out 2>&1 || { tail -20 gpurun_out/r05f_smoke.out; exit 1; }
tail -1 gpurun_out/r05f_smoke.out
timeout -k 10 600 python3 bench.py > gpurun_out/r05f_bench.out 2>&1 || { tail -20 gpurun_out/r05f_bench.out; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r05f_bench.out').read().strip().splitlines()[-1])
r=d['roofline']; print('value',d['value'],'ms',d['ms_per_step'],'kernel',r['kernel_ms_per_launch'],'ceiling',r.get('shape_ceiling_ms'),'k/c',r.get('kernel_over_ceiling'),'step/c',r.get('step_over_ceiling'))
print('per_packet', d.get('per_packet_drop_in'))
for k in ('secondary_order','config3_bridge','config4_lb','nat_random_keys','nat_churn'): print(k, d[k].get('ms_per_step'), d[k].get('kernel_ms_per_launch'), d[k].get('kernel_over_ceiling'), (d[k].get('parity') or {}).get('match'))
"
