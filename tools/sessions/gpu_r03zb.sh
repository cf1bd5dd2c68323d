#!/bin/bash
# write-through fold stamps (default build) vs write-back (VP_WB_FOLD build)
set -o pipefail
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
T=r03zb
WB=$PWD/vigor_amd/wb/libvigpath.so
for v in wt wb wt wb; do
  L=""; [ $v = wb ] && L=$WB
  VIGPATH_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --no-extra --steps 40 > $O/${T}_$v.log 2>&1 || exit $?
  grep '^{' $O/${T}_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'], d['roofline']['kernel_ms_per_launch'], d['parity']['match'])"
done
for v in wt wb; do
  L=""; [ $v = wb ] && L=$WB
  rm -rf $O/${T}_kt_$v
  VIGPATH_LIB=$L timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/${T}_kt_$v -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu --no-e2e --no-extra > $O/${T}_kt_$v.log 2>&1 || exit $?
done
