# Round-1 GPU session p: touch bins (single-pass timestamp fold) for vignat/vigfw.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
rm -rf $O/prof_kt5
timeout -k 10 300 python -u -m pytest tests/test_nat_gpu.py tests/test_fw_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_natfw.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 bench.py --no-cpu > $O/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt5 -- python3 bench.py --steps 10 --warmup 2 --no-cpu > $O/prof_kt5.log 2>&1
rc=$?
tail -15 $O/pytest_natfw.log; tail -3 $O/pytest_gpu.log; cat $O/bench.log
exit $rc
