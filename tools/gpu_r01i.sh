# Round-1 GPU session i: vigfw GPU path + all nf.h shims; full GPU suite; NF side benches.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fw_gpu.py tests/test_nf_shim_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest_fw.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 400 python3 tools/bench_nf.py > $O/bench_nf.log 2>&1
rc=$?
tail -5 $O/pytest_fw.log; tail -3 $O/pytest_gpu.log; cat $O/bench_nf.log
exit $rc
