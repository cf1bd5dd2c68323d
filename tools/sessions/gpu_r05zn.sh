#!/bin/bash
# round 5 session zn: viglb's bins -- default, run words off
# (VIGPATH_BIN_RUNS=0), bins off (VIGPATH_TOUCH_BINS=0), interleaved twice;
# vignat round robin the same way
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
for v in "" "VIGPATH_BIN_RUNS=0" "VIGPATH_TOUCH_BINS=0"; do
env $v timeout -k 10 300 python3 tools/bench_extra.py config4_lb > $O/r05zn_lb.out 2>&1 || { tail -20 $O/r05zn_lb.out; exit 1; }
tail -1 $O/r05zn_lb.out | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['config4_lb']; print('lb [$v]', d['ms_per_step'], d['kernel_ms_per_launch'], d['parity']['match'])"
env $v timeout -k 10 200 python3 bench.py --no-extra --no-cpu --no-e2e > $O/r05zn_rr.json 2>$O/r05zn_rr.err || { tail -20 $O/r05zn_rr.err; exit 1; }
python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print('nat [$v]', d['ms_per_step'], r['kernel_ms_per_launch'])" $O/r05zn_rr.json
done
done
