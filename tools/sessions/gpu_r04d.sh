#!/bin/bash
# round 4 session d: GPU suite (run entries in the touch bins, pipelined
# owner probe), the bench, --route-all, the mbuf probe, a kernel trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/r04d_$name.out" 2> "gpurun_out/r04d_$name.err"
  local rc=$?
  tail -c 1500 "gpurun_out/r04d_$name.out"; echo
  if [ $rc -ne 0 ]; then echo "step $name failed rc=$rc"; tail -30 "gpurun_out/r04d_$name.err"; exit $rc; fi
}
step pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench 700 python -u bench.py
step routeall 300 python -u bench.py --route-all --no-cpu --no-e2e --no-extra --steps 10
step mbufprobe 300 python -u tools/mbuf_probe.py --chunks 1048576,4194304 --blocks 64,256,1024 --variants shuffled,sequential,dense
step trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04d_prof -o run -- python3 bench.py --no-cpu --no-e2e --no-extra --steps 10
