#!/bin/bash
# round 6 session u (diagnostic build): the per-packet drop-in with the
# server's packet work skipped (VIGPATH_SERVE_ECHO: lane 0 answers the WAN port
# at once, frame unchanged) against the real path, twice: the round trip's
# floor and the packet work's share
# (the echo switch lived in a temporary build only; it is not in the tree)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
for i in 1 2; do
  for m in real echo; do
    if [ $m = echo ]; then export VIGPATH_SERVE_ECHO=1; else unset VIGPATH_SERVE_ECHO; fi
    timeout -k 10 300 python3 -c "
import bench, json
print(json.dumps(bench.per_packet_drop_in(batches=(0,))))" > $O/r06u_pp_${m}_$i.json 2> $O/r06u_pp_${m}_$i.err || { tail -20 $O/r06u_pp_${m}_$i.err; exit 1; }
    echo "$m $(cat $O/r06u_pp_${m}_$i.json)"
  done
done
