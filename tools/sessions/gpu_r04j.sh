#!/bin/bash
# round 4 session j: GPU suite (sliced padded exchange written by pass 1,
# host-gather mbuf mode), --route-all, the mbuf probe over modes/threads
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/r04j_$name.out" 2> "gpurun_out/r04j_$name.err"
  local rc=$?
  tail -c 1200 "gpurun_out/r04j_$name.out"; echo
  if [ $rc -ne 0 ]; then echo "step $name failed rc=$rc"; tail -30 "gpurun_out/r04j_$name.err"; exit $rc; fi
}
step shard 300 python -u -m pytest tests/test_shard_gpu.py tests/test_mbuf_gpu.py -x -v --timeout 120 --timeout-method thread
step pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step routeall 300 python -u bench.py --route-all --no-cpu --no-e2e --no-extra --steps 10
VIGPATH_MBUF_THREADS=8 step probe8 300 python -u tools/mbuf_probe.py --modes host,gpu --variants shuffled,dense --chunks 1048576,262144
VIGPATH_MBUF_THREADS=16 step probe16 300 python -u tools/mbuf_probe.py --modes host --variants shuffled --chunks 1048576,262144
