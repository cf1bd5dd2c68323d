#!/bin/bash
# round 5 session b: the N > 1 watchdog on the box.
#  1. two ranks sharing GPU 0 over gloo (VIGPATH_COMM=host), rank 1 stalls
#     400 s in its 4th batch: both watchdogs (budget 20 s) must fire, rank 0
#     prints the partial line, exit status 3 (expected; checked below)
#  2. one rank with a live RCCL communicator (--route-all), stalled 60 s: the
#     watchdog calls vp_comm_abort (ncclCommAbort) on it, exit 3
#  3. the normal two-rank gloo rehearsal: the full line with stages_ms
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --no-cpu --no-e2e --no-extra --steps 5 --warmup 2 --batch 1048576 --flows 1048576"
true || true
VIGPATH_COMM=host VIGPATH_STALL=1:400000:3 VIGPATH_WATCHDOG_S=20 timeout -k 10 200 $B --gpus 2 \
  > gpurun_out/r05b_stall2.out 2> gpurun_out/r05b_stall2.err
rc=$?
echo "stall2 rc=$rc"; grep '^{' gpurun_out/r05b_stall2.out; grep -a "WATCHDOG\|abort" gpurun_out/r05b_stall2.err | head -5
[ $rc -ne 0 ] || exit 1
VIGPATH_STALL=0:60000:3 VIGPATH_WATCHDOG_S=15 timeout -k 10 200 $B --route-all \
  > gpurun_out/r05b_stall_rccl.out 2> gpurun_out/r05b_stall_rccl.err
rc=$?
echo "stall_rccl rc=$rc"; grep '^{' gpurun_out/r05b_stall_rccl.out; grep -a "WATCHDOG\|abort" gpurun_out/r05b_stall_rccl.err | head -5
[ $rc -ne 0 ] || exit 1
rocm-smi --showuse 2>&1 | head -12
VIGPATH_COMM=host timeout -k 10 300 $B --gpus 2 > gpurun_out/r05b_shard2.out 2> gpurun_out/r05b_shard2.err || { tail -20 gpurun_out/r05b_shard2.err; exit 1; }
grep -o '"value": [0-9.]*\|"stages_ms": {"rank0": {[^}]*}' gpurun_out/r05b_shard2.out
