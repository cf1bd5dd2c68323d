#!/bin/bash
# round 5 session d: kernel traces of the chunked owner pipeline (route-all)
# at 2^20 and 2^21 packets per chunk, to see each chunk's pass 1 / probe /
# pass 2 durations and the gaps between them
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for ch in 1048576 2097152; do
  rm -rf gpurun_out/r05d_kt_$ch
  VIGPATH_OWN_CHUNK=$ch timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05d_kt_$ch -- python3 bench.py --route-all --no-cpu --no-e2e --no-extra --steps 3 --warmup 2 > gpurun_out/r05d_kt_$ch.log 2>&1 || { tail -20 gpurun_out/r05d_kt_$ch.log; exit 1; }
done
find gpurun_out/r05d_kt_1048576 -name "*kernel_trace*" | head
