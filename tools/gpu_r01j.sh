# Round-1 GPU session j: touch reduce on its own stream (overlapped), packed pairs, polled read-back.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 bench.py --no-cpu > $O/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt2 -- python3 bench.py --steps 10 --warmup 2 --no-cpu > $O/prof_kt2.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log; cat $O/bench.log
exit $rc
