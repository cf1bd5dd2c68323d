# Round-1 GPU session r: per-GPU rate vs flow-table size (config 5 holds 16M flows per replica).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
: > $O/flows_bench.log
for f in 1048576 2097152 4194304 16777216; do
  timeout -k 10 300 python3 bench.py --flows $f --steps 5 --warmup 2 --no-cpu >> $O/flows_bench.log 2>&1 || exit $?
done
grep '^{' $O/flows_bench.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d['roofline']
    print(d['config']['flows'], d['value'], d['ms_per_step'], r['kernel_ms_per_launch'], r['kernel_mpps'])"
