#!/bin/bash
# round 6 session o: the per-packet server's first poll after an answer
# delayed (VIGPATH_SERVE_AFTER, 10-ns ticks): the per-packet tests at 60, then
# the per-packet drop-in with fixed delays 0 and 45 and the adaptive delay from 0, 45 and 90, twice (answer chunks)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
VIGPATH_SERVE_AFTER=60 timeout -k 10 600 python -u -m pytest tests/test_nat_gpu.py tests/test_nf_shim_gpu.py -x -q --timeout 200 \
  --timeout-method thread -k "process_one or nf_loop or shim" > $O/r06r_pytest.log 2>&1 || { tail -40 $O/r06r_pytest.log; exit 1; }
tail -1 $O/r06r_pytest.log
for i in 1 2; do
for a in 0 45 adapt0 adapt45 adapt90; do
  case $a in adapt*) export VIGPATH_SERVE_ADAPT=1; av=${a#adapt};; *) export VIGPATH_SERVE_ADAPT=0; av=$a;; esac
  VIGPATH_SERVE_AFTER=$av timeout -k 10 300 python3 -c "
import bench, json
print(json.dumps(bench.per_packet_drop_in(batches=(0,))))" > $O/r06r_pp_$a.json 2> $O/r06r_pp_$a.err || { tail -20 $O/r06r_pp_$a.err; exit 1; }
  echo "after=$a $(cat $O/r06r_pp_$a.json)"
done
done
