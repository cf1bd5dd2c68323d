#!/bin/bash
# round 6 session ae: the classify's own control-block publication
# (VIGPATH_TILE_PUB) by arrival mode -- 1 one counter with every block's
# release, 2 the same without the release (timing only), 3 counted per group
# of blocks b % 8 first, 4 as 3 without the stores' wait before the barrier --
# against the fold's (0), headline, interleaved twice
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
for i in 1 2; do
  for p in 0 1 2 3 4; do
    VIGPATH_TILE_PUB=$p timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --no-extra > $O/r06ae_rr_${p}_$i.json 2> $O/r06ae_rr_${p}_$i.err || { tail -20 $O/r06ae_rr_${p}_$i.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print('pub', sys.argv[2], d['value'], d['ms_per_step'], r.get('kernel_ms_per_launch'), r.get('frac_step'), d['parity']['match'])" $O/r06ae_rr_${p}_$i.json $p
  done
done
