set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_nat_gpu.py tests/test_lb_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_natlb.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python3 bench.py > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 python3 tools/ablate.py 5 > gpurun_out/ablate.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_natlb.log; cat gpurun_out/smoke.log gpurun_out/bench.log gpurun_out/ablate.log
exit $rc
