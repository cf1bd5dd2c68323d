#!/bin/bash
# round 4 session ac: vignat tail sums of long mbuf frames from host threads
# (default) against the gather kernel (VIGPATH_MBUF_TAILS=gpu): mbuf tests,
# the bench's end-to-end keys. Host tails measured 26-38 against 87 Mpps IMIX: reverted
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_mbuf_gpu.py tests/test_nf_shim_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ac_pytest.out 2>&1 || { tail -30 gpurun_out/r04ac_pytest.out; exit 1; }
tail -1 gpurun_out/r04ac_pytest.out
for t in gpu host gpu host; do
  VIGPATH_MBUF_TAILS=$t timeout -k 10 400 python3 bench.py --no-cpu --no-extra --steps 5 > gpurun_out/r04ac_bench_$t.out 2>&1 || exit $?
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/r04ac_bench_$t.out') if l.startswith('{')][0])
print('$t', *[(k, d[k]['value'], d[k].get('gbit_per_s'), (d[k].get('parity') or {}).get('match')) for k in ['end_to_end_mbuf','end_to_end_mbuf_imix']])
"
done
