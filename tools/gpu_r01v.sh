# Round-1 GPU session v: re-validate HEAD after the container rebuild; tests, bench, kernel trace, PMC traffic, table-size sweep.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
rm -rf $O/prof_kt7 $O/prof_fetch4 $O/prof_write4
: > $O/flows_bench.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 bench.py > $O/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt7 -- python3 bench.py --steps 10 --warmup 2 --no-cpu > $O/prof_kt7.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_fetch4 -- python3 bench.py --steps 5 --warmup 2 --no-cpu > $O/prof_fetch4.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_write4 -- python3 bench.py --steps 5 --warmup 2 --no-cpu > $O/prof_write4.log 2>&1 && \
for f in 4194304 16777216; do
  timeout -k 10 300 python3 bench.py --flows $f --steps 5 --warmup 2 --no-cpu >> $O/flows_bench.log 2>&1 || exit $?
done
rc=$?
tail -3 $O/pytest_gpu.log; cat $O/bench.log; grep -h '^{' $O/flows_bench.log | cut -c1-400
exit $rc
