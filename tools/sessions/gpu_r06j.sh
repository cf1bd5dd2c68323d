#!/bin/bash
# round 6 session j: the host's side of a steady step (VIGPATH_HOSTPROF=1:
# entry -> classify issued -> fold issued -> control block seen -> exit, per
# call), and vigbridge's PMC traffic (config-3-shaped batches)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
VIGPATH_HOSTPROF=1 timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --no-extra --steps 10 > $O/r06j_hostprof.json 2> $O/r06j_hostprof.err || { tail -20 $O/r06j_hostprof.err; exit 1; }
grep "vigpath hostprof" $O/r06j_hostprof.err | tail -12
bash tools/gpu_session.sh r06j pmcnf:bridge
