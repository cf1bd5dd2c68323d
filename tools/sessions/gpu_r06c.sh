#!/bin/bash
# round 6 session c: vp_process_one's mailbox with tagged request chunks (the
# frame in the poll) and four polls in flight -- the per-packet tests, then
# the per-packet drop-in timing with 1, 2 and 4 polling waves (a request
# claimed by the first wave to see it)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_nat_gpu.py tests/test_nf_shim_gpu.py -x -v --timeout 200 \
  --timeout-method thread -k "process_one or nf_loop or shim or serve" > $O/r06c_pytest.log 2>&1 || { tail -40 $O/r06c_pytest.log; exit 1; }
grep -E "passed|failed" $O/r06c_pytest.log | tail -2
for pp in "1 0" "2 0" "4 0" "2 1" "1 0" "2 0" "4 0"; do set -- $pp; prof=$2; export VIGPATH_SERVE_WAVES=$1
  VIGPATH_SERVE_PROF=$prof timeout -k 10 300 python3 -c "
import bench, json
print(json.dumps(bench.per_packet_drop_in()))" > $O/r06c_pp_$1_$prof.json 2> $O/r06c_pp_$1_$prof.err || { tail -20 $O/r06c_pp_$1_$prof.err; exit 1; }
  cat $O/r06c_pp_$1_$prof.json
done
