set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_nat_gpu.py -q -x > gpurun_out/pytest_nat.log 2>&1 && \
timeout -k 10 300 python3 tools/bench_e2e.py > gpurun_out/bench_e2e.log 2>&1 && \
VIGPATH_HOST_CHUNK=4194304 timeout -k 10 300 python3 tools/bench_e2e.py > gpurun_out/bench_e2e_4m.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_nat.log; cat gpurun_out/bench_e2e.log gpurun_out/bench_e2e_4m.log
exit $rc
