#!/bin/bash
# round 5 session zl: the final build's default bench line, its kernel trace
# and PMC passes (headline), and the uniform order's FETCH/WRITE passes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py > $O/r05zl_bench.json 2> $O/r05zl_bench.err || { tail -20 $O/r05zl_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/r05zl_bench.json').read().strip().splitlines()[-1]); r=d['roofline']
print(d['value'], d['ms_per_step'], r['kernel'], r['kernel_ms_per_launch'], r['frac'], r.get('kernel_over_ceiling'), r.get('traffic'))
print(d.get('per_packet_drop_in',{}).get('per_packet'), d.get('cpu_baseline',{}).get('value'))
for k in ('config4_lb','config3_bridge','nat_random_keys','nat_churn','secondary_order'):
  e=d.get(k) or {}
  print(k, {x: e.get(x) for x in ('value','ms_per_step','kernel_ms_per_launch','frac')}, (e.get('parity') or {}).get('match'))"
bash tools/gpu_session.sh r05zl trace pmc || exit 1
rm -rf $O/r05zl_uni_*
for c in FETCH_SIZE WRITE_SIZE; do
timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $O/r05zl_uni_$c -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-e2e --no-extra --order uniform > $O/r05zl_uni_$c.log 2>&1 || exit 1
done
echo done
