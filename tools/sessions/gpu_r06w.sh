#!/bin/bash
# round 6 session w: the headline's timed loop in C (host/steps.c) against
# the Python loop (VIGPATH_BENCH_PYLOOP=1), interleaved twice
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
for i in 1 2; do
  for p in 0 1; do
    VIGPATH_BENCH_PYLOOP=$p timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --no-extra > $O/r06w_rr_${p}_$i.json 2> $O/r06w_rr_${p}_$i.err || { tail -20 $O/r06w_rr_${p}_$i.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print('pyloop', sys.argv[2], d['value'], d['ms_per_step'], r.get('kernel_ms_per_launch'), r.get('frac'), r.get('frac_step'), r.get('kernel_over_ceiling'), d['parity']['match'])" $O/r06w_rr_${p}_$i.json $p
  done
done
