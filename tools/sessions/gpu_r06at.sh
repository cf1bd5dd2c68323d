#!/bin/bash
# round 6 session at: the per-packet server's stamps through a second wave
# (VIGPATH_SERVE_STAMPER=1, this build's default) against the serving wave's
# own (=0): the per-packet and golden GPU tests with it, then the drop-in
# interleaved five times
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_nat_gpu.py tests/test_nf_shim_gpu.py tests/test_golden.py -x -q -m gpu --timeout 300 \
  --timeout-method thread > $O/r06at_pytest.log 2>&1 || { tail -40 $O/r06at_pytest.log; exit 1; }
tail -1 $O/r06at_pytest.log
for i in 1 2 3 4 5; do
  for v in 1 0; do
    VIGPATH_SERVE_STAMPER=$v timeout -k 10 300 python3 -c "
import bench, json
print(json.dumps(bench.per_packet_drop_in(batches=(0,))))" > $O/r06at_pp_${v}_$i.json 2> $O/r06at_pp_${v}_$i.err || { tail -20 $O/r06at_pp_${v}_$i.err; exit 1; }
    echo "stamper=$v $(cat $O/r06at_pp_${v}_$i.json)"
  done
done
