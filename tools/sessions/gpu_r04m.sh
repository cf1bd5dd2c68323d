#!/bin/bash
# round 4 session m: the random-key workload with 1x / 2x / 4x buckets
# (VIGPATH_SPARSE), reprobes against row locality
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/r04m_$name.out" 2> "gpurun_out/r04m_$name.err"
  local rc=$?
  tail -c 700 "gpurun_out/r04m_$name.out"; echo
  if [ $rc -ne 0 ]; then echo "step $name failed rc=$rc"; tail -30 "gpurun_out/r04m_$name.err"; exit $rc; fi
}
for sp in 0 1 2 1; do
  VIGPATH_SPARSE=$sp step rand_sp$sp 200 python3 tools/bench_extra.py nat_random_keys
done
VIGPATH_SPARSE=1 step churn_sp1 200 python3 tools/bench_extra.py nat_churn
VIGPATH_SPARSE=1 step head_sp1 200 python3 bench.py --no-cpu --no-e2e --no-extra --steps 10
VIGPATH_SPARSE=1 step uni_sp1 200 python3 bench.py --no-cpu --no-e2e --no-extra --steps 10 --order uniform
