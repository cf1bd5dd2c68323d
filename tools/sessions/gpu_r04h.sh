#!/bin/bash
# round 4 session h: SQ counters of the fold kernel (full, and with the
# entry loop skipped: VIGPATH_FOLD_DIAG=1)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -s KILL "$t" "$@" > "gpurun_out/r04h_$name.out" 2> "gpurun_out/r04h_$name.err"
  local rc=$?
  tail -c 200 "gpurun_out/r04h_$name.out"; echo
  if [ $rc -ne 0 ]; then echo "step $name failed rc=$rc"; tail -30 "gpurun_out/r04h_$name.err"; exit $rc; fi
}
rocprofv3 -L > gpurun_out/r04h_counters.txt 2>&1 || true
T="python3 bench.py --no-cpu --no-e2e --no-extra --steps 5 --warmup 1"
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
B="SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
for d in 0 1; do
  VIGPATH_FOLD_DIAG=$d step a$d 150 rocprofv3 --pmc $A --kernel-include-regex touch_bins --output-format csv -d gpurun_out/r04h_a$d -o run -- $T
  VIGPATH_FOLD_DIAG=$d step b$d 150 rocprofv3 --pmc $B --kernel-include-regex touch_bins --output-format csv -d gpurun_out/r04h_b$d -o run -- $T
done
