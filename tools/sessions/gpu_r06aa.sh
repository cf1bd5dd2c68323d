#!/bin/bash
# round 6 session aa: the launch calls' host cost (VIGPATH_HOSTPROF=2, tools/
# hostprof_stats.py) and the headline step under the HIP runtime's kernarg
# placement settings, twice each
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
for i in 1 2; do
  for v in base dev0 dev1 hdp0; do
    unset HIP_FORCE_DEV_KERNARG DEBUG_CLR_KERNARG_HDP_FLUSH_WA
    case $v in dev0) export HIP_FORCE_DEV_KERNARG=0;; dev1) export HIP_FORCE_DEV_KERNARG=1;; hdp0) export DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0;; esac
    VIGPATH_HOSTPROF=2 timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --no-extra > $O/r06aa_${v}_$i.json 2> $O/r06aa_${v}_$i.err || { tail -20 $O/r06aa_${v}_$i.err; exit 1; }
    python3 -c "
import json,sys; sys.path.insert(0,'tools'); import hostprof_stats as H
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print(sys.argv[3], d['value'], d['ms_per_step'], r.get('kernel_ms_per_launch'), r.get('frac_step'), d['parity']['match'], H.summary(H.load(sys.argv[2])))" $O/r06aa_${v}_$i.json $O/r06aa_${v}_$i.err $v
  done
done
