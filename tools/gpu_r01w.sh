# Round-1 GPU session w: cooperative reprobe walk; tests, table-size sweep, bucket sparsity, timeline.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
: > $O/flows_bench.log
rm -rf $O/tl4
timeout -k 10 300 python -u -m pytest tests/test_nat_gpu.py tests/test_fw_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_natfw.log 2>&1 && \
for f in 1048576 4194304 16777216; do
  for sp in 0 1; do
    VIGPATH_SPARSE=$sp timeout -k 10 300 python3 bench.py --flows $f --steps 5 --warmup 2 --no-cpu >> $O/flows_bench.log 2>&1 || exit $?
  done
done && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl4 -o run -- python3 bench.py --flows 4194304 --steps 5 --warmup 2 --no-cpu > $O/tl4.log 2>&1
rc=$?
tail -3 $O/pytest_natfw.log
grep '^{' $O/flows_bench.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d['roofline']
    print(d['config']['flows'], d['value'], d['ms_per_step'], r.get('kernel_ms_per_launch'), r.get('kernel_mpps'))"
python3 tools/step_timeline.py $O/tl4 nat_classify64 1
exit $rc
