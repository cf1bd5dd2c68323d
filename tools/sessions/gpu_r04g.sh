#!/bin/bash
# round 4 session g: the fold's entry loop taken apart (VIGPATH_FOLD_DIAG 4:
# no LDS atomics, 8: no entry loads, 16: no chunk search, 24: neither)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/r04g_$name.out" 2> "gpurun_out/r04g_$name.err"
  local rc=$?
  tail -c 300 "gpurun_out/r04g_$name.out"; echo
  if [ $rc -ne 0 ]; then echo "step $name failed rc=$rc"; tail -30 "gpurun_out/r04g_$name.err"; exit $rc; fi
}
T="python3 bench.py --no-cpu --no-e2e --no-extra --steps 10"
for d in 0 4 8 16 24; do
  VIGPATH_FOLD_DIAG=$d step diag$d 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04g_diag$d -o run -- $T
done
VIGPATH_FOLD_DIAG=16 VIGPATH_FOLD_U=32 step diag16u32 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04g_diag16u32 -o run -- $T
