#!/bin/bash
# round 6 session aj: the per-packet server's late-poll step
# (VIGPATH_SERVE_UP: ticks the first poll's delay grows by after a request it
# missed; 8 the default), 4 / 8 / 16 / 24, interleaved three times
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
for i in 1 2 3; do
  for u in 4 8 16 24; do
    VIGPATH_SERVE_UP=$u timeout -k 10 300 python3 -c "
import bench, json
print(json.dumps(bench.per_packet_drop_in(batches=(0,))))" > $O/r06aj_pp_${u}_$i.json 2> $O/r06aj_pp_${u}_$i.err || { tail -20 $O/r06aj_pp_${u}_$i.err; exit 1; }
    echo "up=$u $(cat $O/r06aj_pp_${u}_$i.json)"
  done
done
