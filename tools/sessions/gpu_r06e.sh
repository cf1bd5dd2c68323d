#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/sessions/gpu_r06d.sh && for w in 2 4; do VIGPATH_SERVE_WAVES=$w timeout -k 10 300 python -u -m pytest tests/test_nat_gpu.py tests/test_nf_shim_gpu.py -x -q --timeout 200 --timeout-method thread -k "process_one or nf_loop" > gpurun_out/r06c_pytest_w$w.log 2>&1 || { tail -30 gpurun_out/r06c_pytest_w$w.log; exit 1; }; tail -1 gpurun_out/r06c_pytest_w$w.log; done && bash tools/sessions/gpu_r06c.sh
