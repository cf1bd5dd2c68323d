#!/bin/bash
# round 4 session c: GPU suite, the bench (defaults), the owner pipeline on
# one GPU (--route-all), 128-byte slots, and a kernel trace of the bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/r04c_$name.out" 2> "gpurun_out/r04c_$name.err"
  local rc=$?
  tail -c 1500 "gpurun_out/r04c_$name.out"; echo
  if [ $rc -ne 0 ]; then echo "step $name failed rc=$rc"; tail -30 "gpurun_out/r04c_$name.err"; exit $rc; fi
}
step mbuf 400 python -u -m pytest tests/test_mbuf_gpu.py -x -v --timeout 120 --timeout-method thread
step pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench 700 python -u bench.py
step routeall 300 python -u bench.py --route-all --no-cpu --no-e2e --no-extra --steps 10
step slot128 300 python -u bench.py --slot 128 --no-cpu --no-e2e --no-extra --steps 10
step trace 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r04c_prof -o run -- python3 bench.py --no-cpu --no-e2e --no-extra --steps 10
