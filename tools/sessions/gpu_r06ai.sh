#!/bin/bash
# round 6 session ai: per-packet drop-in without a hipSetDevice per packet
# (this build) against the last commit's library (build_ab/old through
# LD_LIBRARY_PATH), interleaved four times on one box; the per-packet tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_nat_gpu.py tests/test_nf_shim_gpu.py -x -q --timeout 200 \
  --timeout-method thread -k "process_one or nf_loop or shim" > $O/r06ai_pytest.log 2>&1 || { tail -40 $O/r06ai_pytest.log; exit 1; }
tail -1 $O/r06ai_pytest.log
for i in 1 2 3 4; do
  for v in new old; do
    if [ $v = new ]; then unset LD_LIBRARY_PATH; else export LD_LIBRARY_PATH=$PWD/build_ab/$v; fi
    timeout -k 10 300 python3 -c "
import bench, json
print(json.dumps(bench.per_packet_drop_in(batches=(0,))))" > $O/r06ai_pp_${v}_$i.json 2> $O/r06ai_pp_${v}_$i.err || { tail -20 $O/r06ai_pp_${v}_$i.err; exit 1; }
    echo "$v $(cat $O/r06ai_pp_${v}_$i.json)"
  done
done
