#!/bin/bash
# round 5 session zk: two 1024-thread tiles (nat_classify64w for run traffic,
# nat_classify64ws with staged bin lines otherwise, chosen from the last
# segment's run tiles) -- GPU suite, then rr and uniform against 256-thread
# blocks, twice
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r05zk_pytest.out 2>&1 || { tail -30 $O/r05zk_pytest.out; exit 1; }
tail -1 $O/r05zk_pytest.out
for i in 1 2; do
for w in 4 16; do
for o in rr uniform; do
VIGPATH_BLOCK_WAVES=$w timeout -k 10 200 python3 bench.py --no-extra --no-cpu --no-e2e --order $o > $O/r05zk_${o}_w$w.json 2>$O/r05zk_${o}_w$w.err || { tail -20 $O/r05zk_${o}_w$w.err; exit 1; }
python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print(sys.argv[2], d['value'], d['ms_per_step'], r['kernel_ms_per_launch'])" $O/r05zk_${o}_w$w.json "$o w$w"
done
done
done
