# Round-1 GPU session za: vigpol parity + side bench after the fused stamp.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
rm -rf $O/polprof2
timeout -k 10 300 python -u -m pytest tests/test_pol_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_pol.log 2>&1 && \
timeout -k 10 300 python3 tools/bench_nf.py --only pol --steps 5 --no-cpu > $O/pol_bench2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/polprof2 -o run -- python3 tools/bench_nf.py --only pol --steps 5 --no-cpu > $O/pol_prof2.log 2>&1
rc=$?
tail -2 $O/pytest_pol.log
grep '^{' $O/pol_bench2.log $O/pol_prof2.log
exit $rc
