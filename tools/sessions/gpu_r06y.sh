#!/bin/bash
# round 6 session y: where the headline step's time over its kernel goes --
# the kernel trace of a short headline run with the host's stage times
# recorded absolute (VIGPATH_HOSTPROF=2, printed at exit), to line up
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
rm -rf $O/r06y_kt
VIGPATH_HOSTPROF=2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/r06y_kt -- python3 bench.py --steps 20 --warmup 2 --no-cpu --no-e2e --no-extra > $O/r06y_kt.log 2>&1 || { tail -20 $O/r06y_kt.log; exit 1; }
grep -c "hostprof abs" $O/r06y_kt.log
VIGPATH_HOSTPROF=2 timeout -k 10 300 python3 bench.py --steps 20 --warmup 2 --no-cpu --no-e2e --no-extra > $O/r06y_plain.log 2>&1 || { tail -20 $O/r06y_plain.log; exit 1; }
grep -c "hostprof abs" $O/r06y_plain.log
