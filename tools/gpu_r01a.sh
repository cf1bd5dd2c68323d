set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 tools/flows_sweep.py > gpurun_out/sweep.log 2>&1 && \
timeout -k 10 300 python3 bench.py > gpurun_out/bench.log 2>&1
