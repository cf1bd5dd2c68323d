#!/bin/bash
# round 5 session n: vp_process_one (vignat's persistent per-packet kernel) --
# its parity tests, the per-packet shim tests, then the drop-in timing
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_nat_gpu.py -k "process_one or per_packet" -x -v --timeout 120 --timeout-method thread > gpurun_out/r05n_pytest.out 2>&1 || { tail -40 gpurun_out/r05n_pytest.out; exit 1; }
tail -1 gpurun_out/r05n_pytest.out
timeout -k 10 300 python -u -m pytest tests/test_nf_shim_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05n_shim.out 2>&1 || { tail -40 gpurun_out/r05n_shim.out; exit 1; }
tail -1 gpurun_out/r05n_shim.out
timeout -k 10 200 python3 -c "import bench, json; print(json.dumps(bench.per_packet_drop_in()))" > gpurun_out/r05n_pp.out 2>&1 || { tail -20 gpurun_out/r05n_pp.out; exit 1; }
tail -2 gpurun_out/r05n_pp.out
VIGPATH_SERVE_PROF=1 timeout -k 10 200 python3 -c "import bench, json; print(json.dumps(bench.per_packet_drop_in(batches=(0,))))" > gpurun_out/r05n_pp2.out 2>&1 || { tail -20 gpurun_out/r05n_pp2.out; exit 1; }
tail -3 gpurun_out/r05n_pp2.out
