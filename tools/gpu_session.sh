#!/bin/bash
# One GPU session on the box (run through gpurun), steps chosen by name:
#   bash tools/gpu_session.sh TAG STEP...
# Steps (each under its own time limit, chained: the first failure ends it):
#   tests    pytest -m gpu (one process)          -> gpurun_out/TAG_pytest.log
#   smoke    __graft_entry__.smoke()              -> gpurun_out/TAG_smoke.log
#   bench    python3 bench.py (defaults)          -> gpurun_out/TAG_bench.log
#   trace    rocprofv3 --kernel-trace --stats of bench.py --no-cpu
#                                                 -> gpurun_out/TAG_kt/
#   pmc      two --pmc passes (FETCH_SIZE, WRITE_SIZE) of bench.py --no-cpu
#                                                 -> gpurun_out/TAG_fetch/, TAG_write/
#   pmcnf:NF the two --pmc passes over tools/bench_nf.py --only NF
#   shard2   bench.py --gpus 2 with VIGPATH_COMM=host (ranks share GPU 0)
#   e2e      tools/bench_e2e.py                   -> gpurun_out/TAG_e2e.log
#   slots:S,S,..  bench.py --slot S (wide frames) per slot -> gpurun_out/TAG_slots.log
#   nf       tools/bench_nf.py                    -> gpurun_out/TAG_nf.log
#   test:EXPR  pytest -m gpu -k EXPR
#   probe[:ARG] tools/stream_probe [ARG]          -> gpurun_out/TAG_probe.log
# Extra bench.py arguments for bench/trace/pmc: BENCH_ARGS env.
set -o pipefail
TAG=$1; shift
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
BA=${BENCH_ARGS:-}
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$secs" "$@"
  local rc=$?
  echo "== $name rc=$rc $(date +%T)"
  return $rc
}
for step in "$@"; do
  case $step in
    tests) run tests 900 python -u -m pytest tests -m gpu -x -v --timeout 200 \
             --timeout-method thread > $O/${TAG}_pytest.log 2>&1 || exit $? ;;
    test:*) k=${step#test:}
            run "$step" 600 python -u -m pytest tests -m gpu -x -v --timeout 200 \
             --timeout-method thread -k "$k" > $O/${TAG}_pytest_${k//[^A-Za-z0-9]/_}.log 2>&1 || exit $? ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" \
             > $O/${TAG}_smoke.log 2>&1 || exit $? ;;
    bench) run bench 600 python3 bench.py $BA > $O/${TAG}_bench.log 2>&1 || exit $? ;;
    trace) rm -rf $O/${TAG}_kt
           run trace 400 rocprofv3 --kernel-trace --stats --output-format csv \
             -d $O/${TAG}_kt -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-e2e --no-extra $BA \
             > $O/${TAG}_kt.log 2>&1 || exit $? ;;
    pmc) rm -rf $O/${TAG}_fetch $O/${TAG}_write
         run pmc_fetch 180 rocprofv3 --pmc FETCH_SIZE --output-format csv \
           -d $O/${TAG}_fetch -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-e2e --no-extra $BA \
           > $O/${TAG}_fetch.log 2>&1 || exit $?
         run pmc_write 180 rocprofv3 --pmc WRITE_SIZE --output-format csv \
           -d $O/${TAG}_write -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-e2e --no-extra $BA \
           > $O/${TAG}_write.log 2>&1 || exit $? ;;
    pmcnf:*) nf=${step#pmcnf:}
         rm -rf $O/${TAG}_${nf}_fetch $O/${TAG}_${nf}_write
         run pmcnf_fetch 240 rocprofv3 --pmc FETCH_SIZE --output-format csv \
           -d $O/${TAG}_${nf}_fetch -- python3 tools/bench_nf.py --only $nf --no-cpu --steps 3 \
           > $O/${TAG}_${nf}_fetch.log 2>&1 || exit $?
         run pmcnf_write 240 rocprofv3 --pmc WRITE_SIZE --output-format csv \
           -d $O/${TAG}_${nf}_write -- python3 tools/bench_nf.py --only $nf --no-cpu --steps 3 \
           > $O/${TAG}_${nf}_write.log 2>&1 || exit $? ;;
    shard2) VIGPATH_COMM=host run shard2 600 python3 bench.py --gpus 2 --no-cpu --no-e2e $BA \
             > $O/${TAG}_shard2.log 2>&1 || exit $? ;;
    e2e) run e2e 600 python3 tools/bench_e2e.py > $O/${TAG}_e2e.log 2>&1 || exit $? ;;
    slots:*) for sl in $(echo ${step#slots:} | tr , ' '); do
               run "slot$sl" 300 python3 bench.py --slot $sl --no-cpu --no-e2e --no-extra $BA \
                 >> $O/${TAG}_slots.log 2>&1 || exit $?
             done ;;
    probe|probe:*) a=${step#probe}; a=${a#:}
           run probe 300 tools/stream_probe $a > $O/${TAG}_probe.log 2>&1 || exit $? ;;
    nf) run nf 900 python3 tools/bench_nf.py > $O/${TAG}_nf.log 2>&1 || exit $? ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
