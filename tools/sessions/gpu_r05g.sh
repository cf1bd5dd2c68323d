#!/bin/bash
# round 5 session g: the fold on its own stream (VIGPATH_FOLD_STREAM=1, the
# Measured: the fold stream made the step slower (0.4915-0.4934 ms against
# 0.4765-0.4766 on one stream: the cross-stream event sits on the path to the
# control block the host waits for); reverted.
# new default) against one stream, interleaved; vignat GPU tests with it
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_nat_gpu.py tests/test_golden.py tests/test_layout_gpu.py tests/test_spec_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05g_pytest.out 2>&1 || { tail -30 gpurun_out/r05g_pytest.out; exit 1; }
tail -1 gpurun_out/r05g_pytest.out
B="python3 bench.py --no-cpu --no-e2e --no-extra --steps 20"
for i in 1 2; do
  for fs in 0 1; do
    VIGPATH_FOLD_STREAM=$fs timeout -k 10 200 $B > gpurun_out/r05g_fs${fs}_$i.out 2>&1 || exit 1
    echo "fs=$fs $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*' gpurun_out/r05g_fs${fs}_$i.out | head -3 | tr '\n' ' ')"
  done
done
