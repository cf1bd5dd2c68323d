#!/bin/bash
# round 5 session zf: whole-line bin entries staged in LDS (1024-thread
# blocks, bins_put_staged) -- vignat tests, then uniform order and round
# robin A/B against VIGPATH_BIN_STAGE=0, twice
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_nat_gpu.py -x -q --timeout 100 --timeout-method thread > $O/r05zf_pytest.out 2>&1 || { tail -30 $O/r05zf_pytest.out; exit 1; }
tail -1 $O/r05zf_pytest.out
for i in 1 2; do
for st in 1 0; do
for o in uniform rr; do
VIGPATH_BIN_STAGE=$st timeout -k 10 200 python3 bench.py --no-extra --no-cpu --no-e2e --order $o > $O/r05zf_${o}_s$st.json 2>$O/r05zf_${o}_s$st.err || { tail -20 $O/r05zf_${o}_s$st.err; exit 1; }
python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print(sys.argv[2], d['value'], d['ms_per_step'], r['kernel_ms_per_launch'])" $O/r05zf_${o}_s$st.json "$o stage$st"
done
done
done
