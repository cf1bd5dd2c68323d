#!/bin/bash
# round 5 session x: instruction/wait counters, vignat headline vs viglb
# config4 (why lb_classify64 runs longer on the same bytes), plus viglb's
# FETCH/WRITE passes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
C="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
rm -rf $O/r05x_*
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/r05x_nat_sq -- python3 bench.py --no-extra --no-cpu --no-e2e --steps 3 --warmup 2 > $O/r05x_nat_sq.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/r05x_lb_sq -- python3 tools/bench_extra.py config4_lb --steps 3 > $O/r05x_lb_sq.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/r05x_lb_fetch -- python3 tools/bench_extra.py config4_lb --steps 3 > $O/r05x_lb_fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/r05x_lb_write -- python3 tools/bench_extra.py config4_lb --steps 3 > $O/r05x_lb_write.log 2>&1 || exit 1
echo done
