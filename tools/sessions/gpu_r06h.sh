#!/bin/bash
# round 6 session h: phase B's key-set dedup with plain (L2-cacheable) pre-reads
# instead of device-scope atomic loads -- the vignat tests, then the churn
# workload timed and traced alone
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_nat_gpu.py tests/test_golden.py tests/test_layout_gpu.py -x -q \
  --timeout 200 --timeout-method thread > $O/r06h_pytest.log 2>&1 || { tail -30 $O/r06h_pytest.log; exit 1; }
tail -1 $O/r06h_pytest.log
for i in 1 2; do
  timeout -k 10 300 python3 tools/bench_extra.py nat_churn > $O/r06h_churn_$i.json 2> $O/r06h_churn_$i.err || { tail -20 $O/r06h_churn_$i.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['nat_churn']
print(d['value'], d['ms_per_step'], d['kernel'], d['kernel_ms_per_launch'], d['parity'])" $O/r06h_churn_$i.json
done
rm -rf $O/r06h_kt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r06h_kt -- python3 tools/bench_extra.py nat_churn > $O/r06h_kt.log 2>&1 || { tail -20 $O/r06h_kt.log; exit 1; }
echo traced
