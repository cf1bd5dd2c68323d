#!/bin/bash
# round 6 session ab: tools/dispatch_probe -- a step of two dependent kernels
# (0.4 ms copy, then an epoch write to host memory the host spins on) through
# HIP launches and through AQL packets in an HSA queue of our own (system and
# agent fences): launch calls' host cost and the step's time, twice
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
for i in 1 2; do
  timeout -k 10 120 ./tools/dispatch_probe 40 > $O/r06ab_probe_$i.log 2>&1 || { cat $O/r06ab_probe_$i.log; exit 1; }
  cat $O/r06ab_probe_$i.log
done
