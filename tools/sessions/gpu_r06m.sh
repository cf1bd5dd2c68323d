#!/bin/bash
# round 6 session m: the first-sighting cut (run_batch, FlowTable::fs_hint) --
# the vignat tests (first_sighting_cut among them), golden and layout tests,
# then the churn workload and the headline, each twice
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_nat_gpu.py tests/test_golden.py tests/test_layout_gpu.py tests/test_spec_gpu.py tests/test_mbuf_gpu.py -x -q \
  --timeout 200 --timeout-method thread > $O/r06m_pytest.log 2>&1 || { tail -40 $O/r06m_pytest.log; exit 1; }
tail -1 $O/r06m_pytest.log
for i in 1 2; do
  timeout -k 10 300 python3 tools/bench_extra.py nat_churn > $O/r06m_churn_$i.json 2> $O/r06m_churn_$i.err || { tail -20 $O/r06m_churn_$i.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['nat_churn']
print('churn', d['value'], d['ms_per_step'], d['kernel'], d['kernel_ms_per_launch'], d['parity']['match'], d['parity'].get('state_match'))" $O/r06m_churn_$i.json
  timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --no-extra > $O/r06m_rr_$i.json 2> $O/r06m_rr_$i.err || { tail -20 $O/r06m_rr_$i.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('rr', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'], d['new_flow_mpps'], d['parity']['match'])" $O/r06m_rr_$i.json
done
rm -rf $O/r06m_kt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r06m_kt -- python3 tools/bench_extra.py nat_churn > $O/r06m_kt.log 2>&1 || { tail -20 $O/r06m_kt.log; exit 1; }
echo traced
