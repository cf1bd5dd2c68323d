#!/bin/bash
# round 5 session zq: random keys at one / two / four buckets per index
# (VIGPATH_SPARSE=0/1/2), interleaved twice
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
for sp in 1 0 2; do
VIGPATH_SPARSE=$sp timeout -k 10 300 python3 tools/bench_extra.py nat_random_keys > $O/r05zq_s$sp.out 2>&1 || { tail -20 $O/r05zq_s$sp.out; exit 1; }
tail -1 $O/r05zq_s$sp.out | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['nat_random_keys']; print('sparse $sp', d['value'], d['ms_per_step'], d['kernel_ms_per_launch'], d['parity']['match'])"
done
done
