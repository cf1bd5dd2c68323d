#!/bin/bash
# round 6 session al: bench.py's C step loop against the reference's bench
# digests (tests/test_golden.py::test_c_step_loop_reproduces_bench_shape)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_golden.py -x -v -m gpu --timeout 300 --timeout-method thread \
  -k "bench_shape" > $O/r06al_pytest.log 2>&1 || { tail -40 $O/r06al_pytest.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/r06al_pytest.log | tail -5
