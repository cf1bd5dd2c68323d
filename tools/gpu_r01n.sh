# Round-1 GPU session n: ablations (occupancy, XCD-aware ranges) + PMC traffic of the new classify.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
rm -rf $O/prof_fetch2 $O/prof_write2
timeout -k 10 400 python3 tools/ablate.py 5 > $O/ablate.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_fetch2 -- python3 bench.py --steps 5 --warmup 2 --no-cpu > $O/prof_fetch2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_write2 -- python3 bench.py --steps 5 --warmup 2 --no-cpu > $O/prof_write2.log 2>&1
rc=$?
cat $O/ablate.log
exit $rc
