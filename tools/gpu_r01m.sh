# Round-1 GPU session m: contiguous per-block tiles as default; order sweep; full suite; bench; profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
rm -rf $O/prof_kt4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 tools/order_sweep.py STRIDED > $O/order.log 2>&1 && \
timeout -k 10 300 python3 bench.py > $O/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt4 -- python3 bench.py --steps 10 --warmup 2 --no-cpu > $O/prof_kt4.log 2>&1 && \
timeout -k 10 400 python3 tools/bench_nf.py --no-cpu > $O/bench_nf.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log; cat $O/order.log $O/bench.log $O/bench_nf.log
exit $rc
