#!/bin/bash
# round 4 session i: the mbuf path's host-gather mode (tests in both modes,
# the probe over modes and thread counts)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/r04i_$name.out" 2> "gpurun_out/r04i_$name.err"
  local rc=$?
  tail -c 1500 "gpurun_out/r04i_$name.out"; echo
  if [ $rc -ne 0 ]; then echo "step $name failed rc=$rc"; tail -30 "gpurun_out/r04i_$name.err"; exit $rc; fi
}
step mbuf 400 python -u -m pytest tests/test_mbuf_gpu.py -x -v --timeout 120 --timeout-method thread
VIGPATH_MBUF_THREADS=8 step probe8 400 python -u tools/mbuf_probe.py --modes host,gpu --variants shuffled,dense --chunks 1048576,262144
VIGPATH_MBUF_THREADS=16 step probe16 400 python -u tools/mbuf_probe.py --modes host --variants shuffled --chunks 1048576,262144
