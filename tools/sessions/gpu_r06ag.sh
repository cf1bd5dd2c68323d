#!/bin/bash
# round 6 session ag: the fold with its loads in one round trip and the
# control block's epoch published without an L2 write-back
# (VIGPATH_PUB_RELEASE=1: the release form) -- every GPU test, the headline
# with and without the release interleaved twice, the fold's duration in a
# kernel trace, churn, vigbridge and viglb
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r06ag_pytest.log 2>&1 || { tail -40 $O/r06ag_pytest.log; exit 1; }
tail -1 $O/r06ag_pytest.log
for i in 1 2; do
  for r in 0 1; do
    VIGPATH_PUB_RELEASE=$r timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --no-extra > $O/r06ag_rr_${r}_$i.json 2> $O/r06ag_rr_${r}_$i.err || { tail -20 $O/r06ag_rr_${r}_$i.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print('rel', sys.argv[2], d['value'], d['ms_per_step'], r.get('kernel_ms_per_launch'), r.get('frac_step'), d['parity']['match'])" $O/r06ag_rr_${r}_$i.json $r
  done
done
rm -rf $O/r06ag_kt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r06ag_kt -- python3 bench.py --steps 20 --warmup 2 --no-cpu --no-e2e --no-extra > $O/r06ag_kt.log 2>&1 || { tail -20 $O/r06ag_kt.log; exit 1; }
python3 - <<'PY'
import csv, glob, statistics as st
f = glob.glob('gpurun_out/r06ag_kt/**/*kernel_trace.csv', recursive=True)[0]
d = {}
for r in csv.DictReader(open(f)):
    d.setdefault(r['Kernel_Name'][:40], []).append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k, v in d.items():
    if 'touch' in k or 'nat_classify' in k:
        print(k, len(v), round(st.median(v), 2))
PY
for w in nat_churn config3_bridge config4_lb; do
  timeout -k 10 300 python3 tools/bench_extra.py $w > $O/r06ag_$w.json 2> $O/r06ag_$w.err || { tail -20 $O/r06ag_$w.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])[sys.argv[2]]
print(sys.argv[2], d['value'], d['ms_per_step'], d.get('kernel'), d.get('kernel_ms_per_launch'), d['parity']['match'], d['parity'].get('state_match'))" $O/r06ag_$w.json $w
done
