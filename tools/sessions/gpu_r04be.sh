#!/bin/bash
# round 4 session be (round end, after 128 touch bins with two run words):
# GPU suite,
# smoke, the driver's bench line, kernel trace and PMC passes of the bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_session.sh r04be tests smoke bench || exit $?
tail -1 gpurun_out/r04be_pytest.log
grep '^{' gpurun_out/r04be_bench.log | tail -1 | head -c 600; echo
BENCH_ARGS=--no-extra bash tools/gpu_session.sh r04be trace pmc || exit $?
