#!/bin/bash
# round 6 session v: the per-packet server's probe with its bucket words
# requested together and the home bucket from LDS, the touch stamped behind
# the answer -- the per-packet tests, then the drop-in twice, and once with
# the stage clock
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_nat_gpu.py tests/test_nf_shim_gpu.py -x -q --timeout 200 \
  --timeout-method thread -k "process_one or nf_loop or shim" > $O/r06v_pytest.log 2>&1 || { tail -40 $O/r06v_pytest.log; exit 1; }
tail -1 $O/r06v_pytest.log
for i in 1 2 3; do
  timeout -k 10 300 python3 -c "
import bench, json
print(json.dumps(bench.per_packet_drop_in(batches=(0,))))" > $O/r06v_pp_$i.json 2> $O/r06v_pp_$i.err || { tail -20 $O/r06v_pp_$i.err; exit 1; }
  echo "pp $(cat $O/r06v_pp_$i.json)"
done
VIGPATH_SERVE_PROF=1 timeout -k 10 300 python3 -c "
import bench, json
print(json.dumps(bench.per_packet_drop_in(batches=(0,))))" > $O/r06v_pp_prof.json 2> $O/r06v_pp_prof.err || { tail -20 $O/r06v_pp_prof.err; exit 1; }
echo "prof $(cat $O/r06v_pp_prof.json)"
