#!/bin/bash
# round 6 session d: vigbridge's classify with the next tile's header
# prefetched, the two MAC hashes batched and the row numbers by batched
# ds_bpermute -- the bridge tests, then config 3 twice
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_bridge_gpu.py tests/test_spec_gpu.py tests/test_golden.py -x -q \
  --timeout 200 --timeout-method thread -k "bridge" > $O/r06d_pytest.log 2>&1 || { tail -40 $O/r06d_pytest.log; exit 1; }
tail -1 $O/r06d_pytest.log
for i in 1 2; do
  timeout -k 10 300 python3 tools/bench_extra.py config3_bridge > $O/r06d_bridge_$i.json 2> $O/r06d_bridge_$i.err || { tail -20 $O/r06d_bridge_$i.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['config3_bridge']
print(d['value'], d['ms_per_step'], d['kernel_ms_per_launch'], d['parity']['match'])" $O/r06d_bridge_$i.json
done
