#!/bin/bash
# round 4 session at (round end, after the one-atomic-per-run fold): GPU suite,
# smoke, the driver's bench line, kernel trace and PMC passes of the bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_session.sh r04at tests smoke bench || exit $?
tail -1 gpurun_out/r04at_pytest.log
grep '^{' gpurun_out/r04at_bench.log | tail -1 | head -c 600; echo
BENCH_ARGS=--no-extra bash tools/gpu_session.sh r04at trace pmc || exit $?
