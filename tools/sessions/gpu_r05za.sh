#!/bin/bash
# round 5 session za: random keys' traffic (FETCH/WRITE passes of
# tools/bench_extra.py nat_random_keys) and kernel trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
rm -rf $O/r05za_*
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/r05za_fetch -- python3 tools/bench_extra.py nat_random_keys --steps 3 > $O/r05za_fetch.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/r05za_write -- python3 tools/bench_extra.py nat_random_keys --steps 3 > $O/r05za_write.log 2>&1 || exit 1
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r05za_kt -- python3 tools/bench_extra.py nat_random_keys --steps 5 > $O/r05za_kt.log 2>&1 || exit 1
tail -1 $O/r05za_kt.log | cut -c1-400
