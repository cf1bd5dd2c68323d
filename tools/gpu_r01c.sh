set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 tools/bench_nf.py --no-cpu > gpurun_out/bench_nf.log 2>&1
tail -3 gpurun_out/pytest_gpu.log; cat gpurun_out/bench_nf.log
