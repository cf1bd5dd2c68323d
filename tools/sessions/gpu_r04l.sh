#!/bin/bash
# round 4 session l: viglb storing 48 bytes of rewritten UDP frames
# (VIGPATH_LB_WB48=1) against the whole 64: tests, rate, PMC traffic;
# kernel traces of the random-key and churn workloads
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/r04l_$name.out" 2> "gpurun_out/r04l_$name.err"
  local rc=$?
  tail -c 600 "gpurun_out/r04l_$name.out"; echo
  if [ $rc -ne 0 ]; then echo "step $name failed rc=$rc"; tail -30 "gpurun_out/r04l_$name.err"; exit $rc; fi
}
VIGPATH_LB_WB48=1 step lbtest 300 python -u -m pytest tests/test_lb_gpu.py tests/test_golden.py -x -q --timeout 120 --timeout-method thread
for i in 1 2; do
  VIGPATH_LB_WB48=0 step lb64_$i 200 python -u tools/bench_nf.py --only lb --no-cpu --steps 10
  VIGPATH_LB_WB48=1 step lb48_$i 200 python -u tools/bench_nf.py --only lb --no-cpu --steps 10
done
VIGPATH_LB_WB48=1 step pmcw 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r04l_lb48_write -- python3 tools/bench_nf.py --only lb --no-cpu --steps 3
VIGPATH_LB_WB48=1 step pmcf 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r04l_lb48_fetch -- python3 tools/bench_nf.py --only lb --no-cpu --steps 3
step trace_random 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04l_random_kt -- python3 tools/bench_extra.py nat_random_keys
step trace_churn 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04l_churn_kt -- python3 tools/bench_extra.py nat_churn
