# Round-1 GPU session zb: re-validate HEAD with vigpol; tests, smoke, bench, kernel trace, PMC traffic.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
rm -rf $O/prof_kt8 $O/prof_fetch5 $O/prof_write5
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 bench.py > $O/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt8 -- python3 bench.py --steps 10 --warmup 2 --no-cpu > $O/prof_kt8.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_fetch5 -- python3 bench.py --steps 5 --warmup 2 --no-cpu > $O/prof_fetch5.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_write5 -- python3 bench.py --steps 5 --warmup 2 --no-cpu > $O/prof_write5.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log; cat $O/bench.log; tail -1 $O/smoke.log
exit $rc
