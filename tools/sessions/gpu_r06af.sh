#!/bin/bash
# round 6 session af: the fold with all of a slice's run words loaded beside
# its count -- the vignat and table GPU tests, the headline twice and its
# kernel trace (the fold's duration), churn once
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_nat_gpu.py tests/test_golden.py tests/test_layout_gpu.py tests/test_spec_gpu.py -x -q \
  --timeout 200 --timeout-method thread > $O/r06af_pytest.log 2>&1 || { tail -40 $O/r06af_pytest.log; exit 1; }
tail -1 $O/r06af_pytest.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --no-extra > $O/r06af_rr_$i.json 2> $O/r06af_rr_$i.err || { tail -20 $O/r06af_rr_$i.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print('rr', d['value'], d['ms_per_step'], r.get('kernel_ms_per_launch'), r.get('frac_step'), d['parity']['match'])" $O/r06af_rr_$i.json
done
rm -rf $O/r06af_kt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r06af_kt -- python3 bench.py --steps 20 --warmup 2 --no-cpu --no-e2e --no-extra > $O/r06af_kt.log 2>&1 || { tail -20 $O/r06af_kt.log; exit 1; }
python3 - <<'PY'
import csv, glob, statistics as st
f = glob.glob('gpurun_out/r06af_kt/**/*kernel_trace.csv', recursive=True)[0]
d = {}
for r in csv.DictReader(open(f)):
    d.setdefault(r['Kernel_Name'][:40], []).append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k, v in d.items():
    if 'touch' in k or 'nat_classify' in k:
        print(k, len(v), round(st.median(v), 2))
PY
timeout -k 10 300 python3 tools/bench_extra.py nat_churn > $O/r06af_churn.json 2> $O/r06af_churn.err || { tail -20 $O/r06af_churn.err; exit 1; }
python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['nat_churn']
print('churn', d['value'], d['ms_per_step'], d['kernel'], d['kernel_ms_per_launch'], d['parity']['match'], d['parity'].get('state_match'))" $O/r06af_churn.json
