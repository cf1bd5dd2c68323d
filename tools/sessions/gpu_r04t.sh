#!/bin/bash
# round 4 session t: two-pass mbuf gather (tail sums eight lanes per frame):
# mbuf tests, the bench's end-to-end keys (64 B and IMIX); measured no gain
# (219 / 83 Mpps against 224-227 / 86-87), reverted
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_mbuf_gpu.py tests/test_nf_shim_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04t_pytest.out 2>&1 || { tail -30 gpurun_out/r04t_pytest.out; exit 1; }
tail -2 gpurun_out/r04t_pytest.out
timeout -k 10 400 python3 bench.py --no-cpu --no-extra --steps 5 > gpurun_out/r04t_bench.out 2>&1 || exit $?
python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/r04t_bench.out') if l.startswith('{')][0])
for k in ['end_to_end','end_to_end_mbuf','end_to_end_mbuf_imix']: print(k, d[k]['value'], d[k].get('gbit_per_s'), (d[k].get('parity') or {}).get('match'))
"
