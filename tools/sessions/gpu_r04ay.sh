#!/bin/bash
# round 4 session ay (round end, after the probe walk in the lane and the
# phase-B gather): GPU suite,
# smoke, the driver's bench line, kernel trace and PMC passes of the bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_session.sh r04ay tests smoke bench || exit $?
tail -1 gpurun_out/r04ay_pytest.log
grep '^{' gpurun_out/r04ay_bench.log | tail -1 | head -c 600; echo
BENCH_ARGS=--no-extra bash tools/gpu_session.sh r04ay trace pmc || exit $?
