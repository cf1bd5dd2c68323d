#!/bin/bash
# round 5 session e: the chunked owner pipeline on ONE stream (no concurrent
# probe / pass 2), kernel traces at 2^20 and 2^21 packets per chunk
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for ch in 1048576 2097152; do
  rm -rf gpurun_out/r05e_kt_$ch
  VIGPATH_OWN_ONESTREAM=1 VIGPATH_OWN_CHUNK=$ch timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05e_kt_$ch -- python3 bench.py --route-all --no-cpu --no-e2e --no-extra --steps 3 --warmup 2 > gpurun_out/r05e_kt_$ch.log 2>&1 || { tail -20 gpurun_out/r05e_kt_$ch.log; exit 1; }
  VIGPATH_OWN_ONESTREAM=1 VIGPATH_OWN_CHUNK=$ch timeout -k 10 300 python3 bench.py --route-all --no-cpu --no-e2e --no-extra --steps 10 > gpurun_out/r05e_ra_$ch.out 2>&1 || exit 1
  echo "onestream chunk=$ch $(grep -o '"ms_per_step": [0-9.]*\|"stages_ms": {"rank0": {[^}]*}\|"match": [a-z]*' gpurun_out/r05e_ra_$ch.out | tr '\n' ' ')"
done
