#!/bin/bash
# round 5 session u: frames64_tiles (viglb, vigfw, vigpol) -- batched row
# permutes, unconditional row loads, raised priority for lb/fw; their tests,
# then config4_lb and the NF bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "lb or fw or pol or shim or shard or owner" > gpurun_out/r05u_pytest.out 2>&1 || { tail -40 gpurun_out/r05u_pytest.out; exit 1; }
tail -1 gpurun_out/r05u_pytest.out
for i in 1 2; do
timeout -k 10 300 python3 tools/bench_extra.py config4_lb > gpurun_out/r05u_lb$i.out 2>&1 || { tail -20 gpurun_out/r05u_lb$i.out; exit 1; }
python3 -c "
import json,sys; t=open(sys.argv[1]).read(); d=json.loads(t[t.index('{'):])
print('lb', {x: d.get(x) for x in ('value','ms_per_step','kernel_ms_per_launch','frac','match')})" gpurun_out/r05u_lb$i.out
done
timeout -k 10 400 python3 tools/bench_nf.py --no-cpu > gpurun_out/r05u_nf.out 2>&1 || { tail -20 gpurun_out/r05u_nf.out; exit 1; }
tail -12 gpurun_out/r05u_nf.out
