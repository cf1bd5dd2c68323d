#!/bin/bash
# round 5 session ze: random keys and churn, 256- vs 1024-thread classify
# blocks (VIGPATH_BLOCK_WAVES), same box, interleaved twice
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
for w in 4 16; do
for x in nat_random_keys nat_churn; do
VIGPATH_BLOCK_WAVES=$w timeout -k 10 300 python3 tools/bench_extra.py $x > $O/r05ze_${x}_w$w.out 2>&1 || { tail -20 $O/r05ze_${x}_w$w.out; exit 1; }
tail -1 $O/r05ze_${x}_w$w.out | python3 -c "import json,sys; d=list(json.loads(sys.stdin.read()).values())[0]; print('$x w$w', d['ms_per_step'], d['kernel_ms_per_launch'], d['parity']['match'])"
done
done
done
