#!/bin/bash
# round 5 session r: vp_process_one (persistent per-packet kernel) -- the whole
# GPU suite, then the default bench line (per-packet drop-in included)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05r_pytest.out 2>&1 || { tail -40 gpurun_out/r05r_pytest.out; exit 1; }
tail -1 gpurun_out/r05r_pytest.out
timeout -k 10 600 python3 bench.py > gpurun_out/r05r_bench.json 2> gpurun_out/r05r_bench.err || { tail -20 gpurun_out/r05r_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r05r_bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('per_packet_drop_in'))"
