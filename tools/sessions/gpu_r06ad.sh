#!/bin/bash
# round 6 session ad: per-packet drop-in, this build against the last commit's
# library (build_ab/old) and two variants of this build (build_ab/varA: the
# server's lookup through tbl_probe as before; varC: serve_probe with the
# home bucket's byte tables from global memory), through LD_LIBRARY_PATH,
# interleaved three times on one box
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
for i in 1 2 3; do
  for v in new old varA varC; do
    if [ $v = new ]; then unset LD_LIBRARY_PATH; else export LD_LIBRARY_PATH=$PWD/build_ab/$v; fi
    timeout -k 10 300 python3 -c "
import bench, json
print(json.dumps(bench.per_packet_drop_in(batches=(0,))))" > $O/r06ad_pp_${v}_$i.json 2> $O/r06ad_pp_${v}_$i.err || { tail -20 $O/r06ad_pp_${v}_$i.err; exit 1; }
    echo "$v $(cat $O/r06ad_pp_${v}_$i.json)"
  done
done
