#!/bin/bash
# round 5 session zo: nat_own_probe's row gather as frames64_tiles' (batched
# permutes, unconditional loads) -- owner-mode tests, then --route-all twice
# with its stage times
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_shard_gpu.py -x -q --timeout 300 --timeout-method thread > $O/r05zo_pytest.out 2>&1 || { tail -30 $O/r05zo_pytest.out; exit 1; }
tail -1 $O/r05zo_pytest.out
for i in 1 2; do
timeout -k 10 300 python3 bench.py --route-all --no-cpu --no-e2e --no-extra --steps 10 > $O/r05zo_ra$i.json 2> $O/r05zo_ra$i.err || { tail -20 $O/r05zo_ra$i.err; exit 1; }
python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d.get('stages_ms'))" $O/r05zo_ra$i.json
done
