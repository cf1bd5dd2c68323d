# Round-1 GPU session x: step timelines vs bucket sparsity at 4M / 16M flows.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
rm -rf $O/tlx_*
for cfg in "16777216 1" "16777216 2" "4194304 2"; do
  set -- $cfg
  VIGPATH_SPARSE=$2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tlx_$1_$2 -o run -- python3 bench.py --flows $1 --steps 5 --warmup 2 --no-cpu > $O/tlx_$1_$2.log 2>&1 || exit $?
done
for cfg in "16777216 1" "16777216 2" "4194304 2"; do
  set -- $cfg
  echo "=== flows $1 sparse $2"; grep '^{' $O/tlx_$1_$2.log | cut -c1-200
  python3 tools/step_timeline.py $O/tlx_$1_$2 nat_classify64 1
done
