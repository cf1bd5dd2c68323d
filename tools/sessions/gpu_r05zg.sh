#!/bin/bash
# round 5 session zg: whole GPU suite with staged bin lines; uniform order's
# FETCH/WRITE and L2 passes; the default bench line
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r05zg_pytest.out 2>&1 || { tail -30 $O/r05zg_pytest.out; exit 1; }
tail -1 $O/r05zg_pytest.out
rm -rf $O/r05zg_uni_*
for c in FETCH_SIZE WRITE_SIZE; do
timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $O/r05zg_uni_$c -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-e2e --no-extra --order uniform > $O/r05zg_uni_$c.log 2>&1 || exit 1
done
bash tools/pmc_tcc.sh r05zg_uni --order uniform || exit 1
timeout -k 10 600 python3 bench.py > $O/r05zg_bench.json 2> $O/r05zg_bench.err || { tail -20 $O/r05zg_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/r05zg_bench.json').read().strip().splitlines()[-1]); r=d['roofline']
print(d['value'], d['ms_per_step'], r['kernel'], r['kernel_ms_per_launch'], r['frac'], r.get('kernel_over_ceiling'))
for k in ('config4_lb','config3_bridge','nat_random_keys','nat_churn','secondary_order'):
  e=d.get(k) or {}
  print(k, {x: e.get(x) for x in ('value','ms_per_step','kernel_ms_per_launch','frac')}, (e.get('parity') or {}).get('match'))"
