# Round-1 GPU session u: reprobes on the register path, touches into the bins; tests + table-size sweep.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
: > $O/flows_bench.log
timeout -k 10 300 python -u -m pytest tests/test_nat_gpu.py tests/test_fw_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_natfw.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
for f in 1048576 4194304 16777216; do
  timeout -k 10 300 python3 bench.py --flows $f --steps 5 --warmup 2 --no-cpu >> $O/flows_bench.log 2>&1 || exit $?
done && \
timeout -k 10 300 python3 bench.py --no-cpu > $O/bench.log 2>&1
rc=$?
tail -3 $O/pytest_natfw.log; tail -2 $O/pytest_gpu.log; cat $O/bench.log
grep '^{' $O/flows_bench.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d['roofline']
    print(d['config']['flows'], d['value'], d['ms_per_step'], r.get('kernel_ms_per_launch'), r.get('kernel_mpps'))"
exit $rc
