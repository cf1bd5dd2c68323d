#!/bin/bash
# round 5 session c: the chunked owner pipeline -- sharded parity (gloo ranks
# sharing GPU 0, one-rank RCCL route-all), then bench.py --route-all at three
# chunk sizes against the unchunked pipeline (VIGPATH_OWN_CHUNK=0)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_shard_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/r05c_pytest.out 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/r05c_pytest.out | grep -v "^E " | cut -c1-150
tail -2 gpurun_out/r05c_pytest.out
# (parity failures: go on to the bench; anything else ends the call)
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
B="python3 bench.py --route-all --no-cpu --no-e2e --no-extra --steps 10"
for ch in 0 524288 1048576 2097152; do
  VIGPATH_OWN_CHUNK=$ch timeout -k 10 200 $B > gpurun_out/r05c_ra_$ch.out 2>&1 || { tail -20 gpurun_out/r05c_ra_$ch.out; exit 1; }
  echo "chunk=$ch $(grep -o '"ms_per_step": [0-9.]*\|"stages_ms": {"rank0": {[^}]*}\|"match": [a-z]*' gpurun_out/r05c_ra_$ch.out | tr '\n' ' ')"
done
