#!/bin/bash
# round 5 session zt: owner-mode pass 1 (and, rerun as zt2, pass 2) on the 1024-thread tile -- owner
# tests, then --route-all with its stages, 1024- vs 256-thread, twice
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_shard_gpu.py tests/test_nat_gpu.py -x -q --timeout 300 --timeout-method thread > $O/r05zt_pytest.out 2>&1 || { tail -30 $O/r05zt_pytest.out; exit 1; }
tail -1 $O/r05zt_pytest.out
for i in 1 2; do
for w in 16 4; do
VIGPATH_BLOCK_WAVES=$w timeout -k 10 300 python3 bench.py --route-all --no-cpu --no-e2e --no-extra --steps 10 > $O/r05zt_ra_w$w.json 2> $O/r05zt_ra_w$w.err || { tail -20 $O/r05zt_ra_w$w.err; exit 1; }
python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); st=d.get('stages_ms',{}).get('rank0',{})
print(sys.argv[2], d['value'], d['ms_per_step'], {k: st.get(k) for k in ('pass1','probe','pass2','fold')})" $O/r05zt_ra_w$w.json "route-all w$w"
done
done
