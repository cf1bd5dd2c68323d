#!/bin/bash
# round 5 session zm: viglb with and without the raised issue priority
# (VIGPATH_PRIO=0), config4_lb interleaved, three times (rerun: the first run shadowed the segment start)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do
for pr in 1 0; do
VIGPATH_PRIO=$pr timeout -k 10 300 python3 tools/bench_extra.py config4_lb > $O/r05zm_lb_p$pr.out 2>&1 || { tail -20 $O/r05zm_lb_p$pr.out; exit 1; }
tail -1 $O/r05zm_lb_p$pr.out | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['config4_lb']; print('prio$pr', d['ms_per_step'], d['kernel_ms_per_launch'], d['frac'], d['parity']['match'])"
done
done
