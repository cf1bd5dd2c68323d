#!/bin/bash
# round 6 session x: the per-packet server with the touch stamped last (after
# the answer word and its clock) -- the per-packet tests, the drop-in three
# times, once with the stage clock; then the headline's C loop against the
# Python loop (session w's A/B)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_nat_gpu.py tests/test_nf_shim_gpu.py -x -q --timeout 200 \
  --timeout-method thread -k "process_one or nf_loop or shim" > $O/r06x_pytest.log 2>&1 || { tail -40 $O/r06x_pytest.log; exit 1; }
tail -1 $O/r06x_pytest.log
for i in 1 2 3; do
  timeout -k 10 300 python3 -c "
import bench, json
print(json.dumps(bench.per_packet_drop_in(batches=(0,))))" > $O/r06x_pp_$i.json 2> $O/r06x_pp_$i.err || { tail -20 $O/r06x_pp_$i.err; exit 1; }
  echo "pp $(cat $O/r06x_pp_$i.json)"
done
VIGPATH_SERVE_PROF=1 timeout -k 10 300 python3 -c "
import bench, json
print(json.dumps(bench.per_packet_drop_in(batches=(0,))))" > $O/r06x_pp_prof.json 2> $O/r06x_pp_prof.err || { tail -20 $O/r06x_pp_prof.err; exit 1; }
echo "prof $(cat $O/r06x_pp_prof.json)"
bash tools/sessions/gpu_r06w.sh
