# Round-1 GPU session zg: final re-validation of HEAD; tests, smoke, bench, kernel trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
rm -rf $O/prof_kt9 $O/prof_fetch6 $O/prof_write6
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 bench.py > $O/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt9 -- python3 bench.py --steps 10 --warmup 2 --no-cpu > $O/prof_kt9.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log; cat $O/bench.log; tail -1 $O/smoke.log
exit $rc
