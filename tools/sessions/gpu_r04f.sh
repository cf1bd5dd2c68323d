#!/bin/bash
# round 4 session f: where the fold's time goes (VIGPATH_FOLD_DIAG: 1 no
# entries, 2 no stamp writes; VIGPATH_FOLD_U 32), each under a kernel trace;
# the mbuf probe on a 2 MB page pool
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/r04f_$name.out" 2> "gpurun_out/r04f_$name.err"
  local rc=$?
  tail -c 600 "gpurun_out/r04f_$name.out"; echo
  if [ $rc -ne 0 ]; then echo "step $name failed rc=$rc"; tail -30 "gpurun_out/r04f_$name.err"; exit $rc; fi
}
T="python3 bench.py --no-cpu --no-e2e --no-extra --steps 10"
for d in 0 1 2 3; do
  VIGPATH_FOLD_DIAG=$d step diag$d 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04f_diag$d -o run -- $T
done
VIGPATH_FOLD_U=32 step u32 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04f_u32 -o run -- $T
VIGPATH_BIN_RUNS=1 VIGPATH_FOLD_U=32 step runs_u32 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04f_runs_u32 -o run -- $T
step mbufprobe 600 python -u tools/mbuf_probe.py --pools huge,pinned --variants shuffled,dense --chunks 1048576,262144 --blocks 256 --streams 2,1
