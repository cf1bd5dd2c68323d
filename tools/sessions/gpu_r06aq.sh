#!/bin/bash
# round 6 session aq: the per-packet server's LDS bucket cache (ServeRows,
# VIGPATH_SERVE_ROWS=1, the default of this build) against none (=0): the
# per-packet tests with it, then the drop-in interleaved four times
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_nat_gpu.py tests/test_nf_shim_gpu.py -x -q --timeout 200 \
  --timeout-method thread -k "process_one or nf_loop or shim" > $O/r06aq_pytest.log 2>&1 || { tail -40 $O/r06aq_pytest.log; exit 1; }
tail -1 $O/r06aq_pytest.log
for i in 1 2 3 4; do
  for r in 1 0; do
    VIGPATH_SERVE_ROWS=$r timeout -k 10 300 python3 -c "
import bench, json
print(json.dumps(bench.per_packet_drop_in(batches=(0,))))" > $O/r06aq_pp_${r}_$i.json 2> $O/r06aq_pp_${r}_$i.err || { tail -20 $O/r06aq_pp_${r}_$i.err; exit 1; }
    echo "rows=$r $(cat $O/r06aq_pp_${r}_$i.json)"
  done
done
