#!/bin/bash
# round 4 session ao (round end): GPU suite, smoke, the driver's bench line,
# kernel trace and PMC passes of the bench; then the 128-byte slot shape's
# memory ceiling and viglb's traffic on config4_lb (session an)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_session.sh r04ao tests smoke bench || exit $?
tail -1 gpurun_out/r04ao_pytest.log
grep '^{' gpurun_out/r04ao_bench.log | tail -1 | head -c 600; echo
BENCH_ARGS=--no-extra bash tools/gpu_session.sh r04ao trace pmc || exit $?
bash tools/sessions/gpu_r04an.sh
