#!/bin/bash
# round 4 session an: the 128-byte slot shape's memory ceiling
# (tools/slot_probe), then HBM traffic of viglb's classify on the bench
# line's config4_lb workload (2^24 packets per launch)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 tools/slot_probe > gpurun_out/r04an_slot_probe.txt 2>&1 || { cat gpurun_out/r04an_slot_probe.txt; exit 1; }
cat gpurun_out/r04an_slot_probe.txt
T="python3 tools/bench_extra.py config4_lb --steps 5"
rm -rf gpurun_out/r04an_lb_fetch gpurun_out/r04an_lb_write
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r04an_lb_fetch -- $T > gpurun_out/r04an_lb_fetch.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r04an_lb_write -- $T > gpurun_out/r04an_lb_write.log 2>&1 || exit $?
tail -c 300 gpurun_out/r04an_lb_write.log
