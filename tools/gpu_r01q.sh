# Round-1 GPU session q: faster bins fold; tests, bench, kernel trace, PMC traffic.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
rm -rf $O/prof_kt6 $O/prof_fetch3 $O/prof_write3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 bench.py > $O/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt6 -- python3 bench.py --steps 10 --warmup 2 --no-cpu > $O/prof_kt6.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_fetch3 -- python3 bench.py --steps 5 --warmup 2 --no-cpu > $O/prof_fetch3.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_write3 -- python3 bench.py --steps 5 --warmup 2 --no-cpu > $O/prof_write3.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log; cat $O/bench.log
exit $rc
