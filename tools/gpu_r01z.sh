# Round-1 GPU session z: vigpol side bench + kernel-trace summary.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
rm -rf $O/polprof
timeout -k 10 300 python3 tools/bench_nf.py --only pol --steps 5 > $O/pol_bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/polprof -o run -- python3 tools/bench_nf.py --only pol --steps 5 --no-cpu > $O/pol_prof.log 2>&1
rc=$?
grep '^{' $O/pol_bench.log $O/pol_prof.log
f=$(find $O/polprof -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && cut -d, -f1-8 "$f" | head -20
exit $rc
