#!/bin/bash
# round 6 session t: the per-packet server's stage clock with the shader clock
# beside it (VIGPATH_SERVE_PROF=1: s_memtime over the packet stage), twice
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
for i in 1 2; do
  VIGPATH_SERVE_PROF=1 timeout -k 10 300 python3 -c "
import bench, json
print(json.dumps(bench.per_packet_drop_in(batches=(0,))))" > $O/r06t_pp_$i.json 2> $O/r06t_pp_$i.err || { tail -20 $O/r06t_pp_$i.err; exit 1; }
  cat $O/r06t_pp_$i.json
done
