#!/bin/bash
# round 5 session p: vp_process_one with the register path and 16-byte system-coherent (was o: no fences,
# loads/stores for the mailbox) -- parity, then the drop-in timing with the
# stage clock, fences off and on
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_nat_gpu.py -k "process_one or per_packet" -x -v --timeout 120 --timeout-method thread > gpurun_out/r05p_pytest.out 2>&1 || { tail -40 gpurun_out/r05p_pytest.out; exit 1; }
tail -1 gpurun_out/r05p_pytest.out
timeout -k 10 300 python -u -m pytest tests/test_nf_shim_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05p_shim.out 2>&1 || { tail -40 gpurun_out/r05p_shim.out; exit 1; }
tail -1 gpurun_out/r05p_shim.out
for f in 0 1 0; do
VIGPATH_SERVE_FENCES=$f VIGPATH_SERVE_PROF=1 timeout -k 10 200 python3 -c "import bench, json; print(json.dumps(bench.per_packet_drop_in(batches=(0,))))" > gpurun_out/r05p_pp$f.out 2>&1 || { tail -20 gpurun_out/r05p_pp$f.out; exit 1; }
echo "fences=$f"; tail -1 gpurun_out/r05p_pp$f.out
done
timeout -k 10 200 python3 -c "import bench, json; print(json.dumps(bench.per_packet_drop_in()))" > gpurun_out/r05p_pp.out 2>&1 || { tail -20 gpurun_out/r05p_pp.out; exit 1; }
tail -1 gpurun_out/r05p_pp.out
