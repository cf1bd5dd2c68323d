#!/bin/bash
# round 4 session ad: the owner probe's per-tile slice check (shard tests,
# --route-all twice), viglb PMC traffic after the run words
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_shard_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ad_pytest.out 2>&1 || { tail -30 gpurun_out/r04ad_pytest.out; exit 1; }
tail -1 gpurun_out/r04ad_pytest.out
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --route-all --no-cpu --no-e2e --no-extra --steps 10 > gpurun_out/r04ad_routeall$i.out 2>&1 || exit $?
  grep -o '"ms_per_step": [0-9.]*\|"probe": [0-9.]*' gpurun_out/r04ad_routeall$i.out | head -2 | tr '\n' ' '; echo
done
bash tools/gpu_session.sh r04ad pmcnf:lb || exit $?
