#!/bin/bash
# round 4 session b: mbuf parity tests, the whole GPU suite, then the bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_mbuf_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r04b_mbuf.log 2>&1 || { echo "mbuf tests failed"; tail -40 gpurun_out/r04b_mbuf.log; exit 1; }
tail -3 gpurun_out/r04b_mbuf.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04b_pytest.log 2>&1 || { echo "gpu suite failed"; tail -30 gpurun_out/r04b_pytest.log; exit 1; }
tail -3 gpurun_out/r04b_pytest.log
timeout -k 10 600 python -u bench.py > gpurun_out/r04b_bench.json 2> gpurun_out/r04b_bench.err
rc=$?
tail -c 3000 gpurun_out/r04b_bench.json
exit $rc
