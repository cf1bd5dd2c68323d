#!/bin/bash
# write-through metadata stores (touch-bin entries, out ports, fold stamps)
# vs write-back (VIGPATH_LIB=vigor_amd/wb/libvigpath.so, built -DVP_WB_META)
set -o pipefail
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
T=r03w
WB=$PWD/vigor_amd/wb/libvigpath.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/${T}_pytest.log 2>&1 || exit $?
tail -1 $O/${T}_pytest.log
for v in wt wb wt wb; do
  L=""; [ $v = wb ] && L=$WB
  VIGPATH_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --no-extra --steps 40 > $O/${T}_$v.log 2>&1 || exit $?
  grep '^{' $O/${T}_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'], d['roofline']['kernel_ms_per_launch'], d['parity']['match'])"
done
for v in wt wb; do
  L=""; [ $v = wb ] && L=$WB
  VIGPATH_LIB=$L timeout -k 10 400 python3 tools/bench_nf.py --only bridge,lb,fw,pol --no-cpu > $O/${T}_nf_$v.log 2>&1 || exit $?
  grep '^{' $O/${T}_nf_$v.log | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('$v', d['config'].get('workload','')[:30] if isinstance(d.get('config'),dict) else '', d['value'], d.get('kernel_mpps'))"
done
for v in wt wb; do
  L=""; [ $v = wb ] && L=$WB
  rm -rf $O/${T}_kt_$v
  VIGPATH_LIB=$L timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/${T}_kt_$v -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu --no-e2e --no-extra > $O/${T}_kt_$v.log 2>&1 || exit $?
done
