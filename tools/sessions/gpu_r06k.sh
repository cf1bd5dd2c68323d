#!/bin/bash
# round 6 session k: where the first (all-new-flows) batch's 17 ms go --
# HIP API and kernel trace of a short headline run
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
rm -rf $O/r06k_ht
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $O/r06k_ht -- python3 bench.py --steps 2 --warmup 2 --no-cpu --no-e2e --no-extra > $O/r06k_ht.log 2>&1 || { tail -20 $O/r06k_ht.log; exit 1; }
ls -R $O/r06k_ht | head
VIGPATH_HOSTPROF=1 timeout -k 10 300 python3 bench.py --steps 2 --warmup 2 --no-cpu --no-e2e --no-extra > $O/r06k_hp.json 2> $O/r06k_hp.err || { tail -20 $O/r06k_hp.err; exit 1; }
grep hostprof $O/r06k_hp.err | head -4
