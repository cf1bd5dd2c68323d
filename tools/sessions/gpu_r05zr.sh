#!/bin/bash
# round 5 session zr: bin count with staged bin lines -- uniform order and
# round robin at 64 / 128 / 256 bins (VIGPATH_BIN_BITS=6/7/8), interleaved
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
for bb in 7 6 8; do
for o in uniform rr; do
VIGPATH_BIN_BITS=$bb timeout -k 10 200 python3 bench.py --no-extra --no-cpu --no-e2e --order $o > $O/r05zr.json 2>$O/r05zr.err || { tail -20 $O/r05zr.err; exit 1; }
python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print(sys.argv[2], d['value'], d['ms_per_step'], r['kernel_ms_per_launch'])" $O/r05zr.json "$o bins2^$bb"
done
done
done
