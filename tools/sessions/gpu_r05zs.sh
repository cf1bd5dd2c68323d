#!/bin/bash
# round 5 session zs: 16M flows on one GPU (config 5's table per rank),
# 1024- vs 256-thread classify blocks, interleaved twice
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
for w in 16 4; do
VIGPATH_BLOCK_WAVES=$w timeout -k 10 300 python3 bench.py --flows 16777216 --no-extra --no-cpu --no-e2e > $O/r05zs.json 2>$O/r05zs.err || { tail -20 $O/r05zs.err; exit 1; }
python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print(sys.argv[2], d['value'], d['ms_per_step'], r['kernel_ms_per_launch'], (d.get('parity') or {}).get('match') if isinstance(d.get('parity'),dict) else d.get('parity'))" $O/r05zs.json "16M w$w"
done
done
