#!/bin/bash
# round 6 session ar: the final tree's per-packet drop-in ten times on one
# box (its spread), after the per-packet and golden tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_nat_gpu.py tests/test_nf_shim_gpu.py tests/test_golden.py -x -q -m gpu --timeout 300 \
  --timeout-method thread > $O/r06ar_pytest.log 2>&1 || { tail -40 $O/r06ar_pytest.log; exit 1; }
tail -1 $O/r06ar_pytest.log
for i in 1 2 3 4 5 6 7 8 9 10; do
  timeout -k 10 300 python3 -c "
import bench, json
print(json.dumps(bench.per_packet_drop_in(batches=(0,))))" > $O/r06ar_pp_$i.json 2> $O/r06ar_pp_$i.err || { tail -20 $O/r06ar_pp_$i.err; exit 1; }
  echo "pp $(cat $O/r06ar_pp_$i.json)"
done
