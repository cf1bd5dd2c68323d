#!/bin/bash
# round 6 session as (diagnostic): the per-packet drop-in with the server's
# flow-table stamps (ts/tseq stores) removed (build_ab/nostamp, a build not
# kept: the table's timestamps go stale) against the real path, through
# LD_LIBRARY_PATH, interleaved five times -- what the stamps' stores cost a
# packet
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
for i in 1 2 3 4 5; do
  for v in new nostamp; do
    if [ $v = new ]; then unset LD_LIBRARY_PATH; else export LD_LIBRARY_PATH=$PWD/build_ab/$v; fi
    timeout -k 10 300 python3 -c "
import bench, json
print(json.dumps(bench.per_packet_drop_in(batches=(0,))))" > $O/r06as_pp_${v}_$i.json 2> $O/r06as_pp_${v}_$i.err || { tail -20 $O/r06as_pp_${v}_$i.err; exit 1; }
    echo "$v $(cat $O/r06as_pp_${v}_$i.json)"
  done
done
