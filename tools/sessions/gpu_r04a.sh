#!/bin/bash
# round 4 session a: the mbuf path's parity tests, then the whole GPU suite
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_mbuf_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r04a_mbuf.log 2>&1 || { echo "mbuf tests failed"; tail -40 gpurun_out/r04a_mbuf.log; exit 1; }
tail -3 gpurun_out/r04a_mbuf.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04a_pytest.log 2>&1
rc=$?
tail -5 gpurun_out/r04a_pytest.log
exit $rc
