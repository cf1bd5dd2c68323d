# Round-1 GPU session h: full GPU suite, bench, kernel-trace + PMC profiles of
# the bench, row-granularity microbenchmark.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 bench.py > $O/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -- python3 bench.py --steps 10 --warmup 2 --no-cpu > $O/prof_kt.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_fetch -- python3 bench.py --steps 5 --warmup 2 --no-cpu > $O/prof_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_write -- python3 bench.py --steps 5 --warmup 2 --no-cpu > $O/prof_write.log 2>&1 && \
timeout -k 10 120 ./tools/gran_probe > $O/gran.log 2>&1
rc=$?
timeout -k 5 60 rocprofv3 -L > $O/counters_list.txt 2>&1
tail -3 $O/pytest_gpu.log; cat $O/bench.log $O/gran.log; tail -3 $O/prof_kt.log
exit $rc
