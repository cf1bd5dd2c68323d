#!/bin/bash
# round 4 session e: run entries in the touch bins on/off/non-temporal (A/B
# on one box, plain and under a kernel trace), the mbuf probe with a 2 MB
# page pool
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/r04e_$name.out" 2> "gpurun_out/r04e_$name.err"
  local rc=$?
  tail -c 1200 "gpurun_out/r04e_$name.out"; echo
  if [ $rc -ne 0 ]; then echo "step $name failed rc=$rc"; tail -30 "gpurun_out/r04e_$name.err"; exit $rc; fi
}
B="python -u bench.py --no-cpu --no-e2e --no-extra --steps 10"
VIGPATH_BIN_RUNS=0 step runs0 200 $B
VIGPATH_BIN_RUNS=1 step runs1 200 $B
VIGPATH_BIN_RUNS=2 step runs2 200 $B
VIGPATH_BIN_RUNS=0 step runs0b 200 $B
VIGPATH_BIN_RUNS=1 step runs1b 200 $B
VIGPATH_BIN_RUNS=0 step trace0 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04e_prof0 -o run -- python3 bench.py --no-cpu --no-e2e --no-extra --steps 10
VIGPATH_BIN_RUNS=1 step trace1 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04e_prof1 -o run -- python3 bench.py --no-cpu --no-e2e --no-extra --steps 10
step mbufprobe 500 python -u tools/mbuf_probe.py --pools pinned,huge --variants shuffled,dense --chunks 524288,1048576 --blocks 256,1024
