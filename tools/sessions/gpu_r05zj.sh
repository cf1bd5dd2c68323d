#!/bin/bash
# round 5 session zj: round robin, 256- vs 1024-thread blocks in the build
# with staged bin lines (does the staging code cost round robin?), twice
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
for w in 4 16; do
VIGPATH_BLOCK_WAVES=$w timeout -k 10 200 python3 bench.py --no-extra --no-cpu --no-e2e > $O/r05zj_w$w.json 2>$O/r05zj_w$w.err || { tail -20 $O/r05zj_w$w.err; exit 1; }
python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print(sys.argv[2], d['value'], d['ms_per_step'], r['kernel_ms_per_launch'], r.get('shape_ceiling_ms'))" $O/r05zj_w$w.json "rr w$w"
done
done
