# Round-1 GPU session v: step timeline at 4M and 16M flows.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
rm -rf $O/tl4 $O/tl16
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl4 -o run -- python3 bench.py --flows 4194304 --steps 5 --warmup 2 --no-cpu > $O/tl4.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl16 -o run -- python3 bench.py --flows 16777216 --steps 5 --warmup 2 --no-cpu > $O/tl16.log 2>&1
rc=$?
python3 tools/step_timeline.py $O/tl4 nat_classify64 2; python3 tools/step_timeline.py $O/tl16 nat_classify64 2
exit $rc
