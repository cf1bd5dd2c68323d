#!/bin/bash
# round 6 session z: per-packet drop-in, this build against the last commit's
# library (build_ab/libvigpath.so through LD_LIBRARY_PATH: the nf.h shim's
# RUNPATH yields to it), interleaved three times on one box
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
for i in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then export LD_LIBRARY_PATH=$PWD/build_ab/old; else unset LD_LIBRARY_PATH; fi
    timeout -k 10 300 python3 -c "
import bench, json
print(json.dumps(bench.per_packet_drop_in(batches=(0,))))" > $O/r06z_pp_${v}_$i.json 2> $O/r06z_pp_${v}_$i.err || { tail -20 $O/r06z_pp_${v}_$i.err; exit 1; }
    echo "$v $(cat $O/r06z_pp_${v}_$i.json)"
  done
done
