#!/bin/bash
# round 5 session zb: one 1024-thread classify block per CU
# (VIGPATH_BLOCK_WAVES=16), rerun with eight run words per block and bin -- vignat tests under it (and the whole suite at the default), then uniform order and
# round robin A/B against the 256-thread blocks
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r05zb_pytest_all.out 2>&1 || { tail -30 $O/r05zb_pytest_all.out; exit 1; }
tail -1 $O/r05zb_pytest_all.out
VIGPATH_BLOCK_WAVES=16 timeout -k 10 600 python -u -m pytest tests/test_nat_gpu.py -x -q --timeout 200 --timeout-method thread > $O/r05zb_pytest.out 2>&1 || { tail -30 $O/r05zb_pytest.out; exit 1; }
tail -1 $O/r05zb_pytest.out
for i in 1 2; do
for w in 4 16; do
for o in uniform rr; do
VIGPATH_BLOCK_WAVES=$w timeout -k 10 300 python3 bench.py --no-extra --no-cpu --no-e2e --order $o > $O/r05zb_${o}_w$w.json 2>$O/r05zb_${o}_w$w.err || { tail -20 $O/r05zb_${o}_w$w.err; exit 1; }
python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print(sys.argv[2], d['value'], d['ms_per_step'], r['kernel_ms_per_launch'], d.get('parity',{}).get('match') if isinstance(d.get('parity'),dict) else d.get('parity'))" $O/r05zb_${o}_w$w.json "$o w$w"
done
done
done
