#!/bin/bash
# round 4 session n: GPU suite, smoke and the bench with two buckets per
# index; the mbuf probe with whole-line write-backs
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_session.sh r04n tests smoke bench || exit $?
timeout -k 10 300 python3 tools/mbuf_probe.py --variants shuffled,dense > gpurun_out/r04n_probe.out 2>&1 &&
timeout -k 10 300 python3 tools/mbuf_probe.py --variants shuffled,dense --lines >> gpurun_out/r04n_probe.out 2>&1
rc=$?; grep '^{' gpurun_out/r04n_probe.out; exit $rc
