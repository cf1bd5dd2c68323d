# Round-1 GPU session k: packed touch reduce (span-walking pass 3), polled read-back.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
rm -rf $O/prof_kt3
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_nat.log 2>&1 && \
timeout -k 10 300 python3 bench.py --no-cpu > $O/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt3 -- python3 bench.py --steps 10 --warmup 2 --no-cpu > $O/prof_kt3.log 2>&1
rc=$?
tail -3 $O/pytest_nat.log; cat $O/bench.log
exit $rc
