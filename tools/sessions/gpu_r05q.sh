#!/bin/bash
# round 5 session q: vp_process_one -- the time read with the frame's first
# chunk; stage clock per load cache policy (0 sc0|sc1, 1 plain, 2 sc1, 3 sc0)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_nat_gpu.py -k "process_one or per_packet" -x -v --timeout 120 --timeout-method thread > gpurun_out/r05q_pytest.out 2>&1 || { tail -40 gpurun_out/r05q_pytest.out; exit 1; }
tail -1 gpurun_out/r05q_pytest.out
timeout -k 10 300 python -u -m pytest tests/test_nf_shim_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05q_shim.out 2>&1 || { tail -40 gpurun_out/r05q_shim.out; exit 1; }
tail -1 gpurun_out/r05q_shim.out
for f in 0 1 2 3 0; do
VIGPATH_SERVE_LPOL=$f VIGPATH_SERVE_PROF=1 timeout -k 10 200 python3 -c "import bench, json; print(json.dumps(bench.per_packet_drop_in(batches=(0,))))" > gpurun_out/r05q_pp$f.out 2>&1 || { tail -20 gpurun_out/r05q_pp$f.out; exit 1; }
echo "lpol=$f"; tail -1 gpurun_out/r05q_pp$f.out
done
