# Round-1 GPU session o: ablation table only (env applied per launch).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 tools/ablate.py 5 > gpurun_out/ablate.log 2>&1
rc=$?
cat gpurun_out/ablate.log
exit $rc
