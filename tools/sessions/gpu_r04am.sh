#!/bin/bash
# round 4 session am: SQ counters of the vignat classify kernels at 64- and
# 128-byte slots (is the tile loop issue-bound?)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -s KILL "$t" "$@" > "gpurun_out/r04am_$name.out" 2> "gpurun_out/r04am_$name.err"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "step $name failed rc=$rc"; tail -30 "gpurun_out/r04am_$name.err"; exit $rc; fi
}
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU"
B="SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
for sl in 64 128; do
  T="python3 bench.py --no-cpu --no-e2e --no-extra --steps 3 --warmup 1 --slot $sl"
  step a$sl 120 rocprofv3 --pmc $A --kernel-include-regex nat_classify --output-format csv -d gpurun_out/r04am_a$sl -o run -- $T
  step b$sl 120 rocprofv3 --pmc $B --kernel-include-regex nat_classify --output-format csv -d gpurun_out/r04am_b$sl -o run -- $T
done
echo done
