# Round-1 GPU session t: reprobe deferral (full home buckets leave the wave); tests + size sweep.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
export SWEEP_FLOWS=1048576,4194304,8388608,16777216
timeout -k 10 300 python -u -m pytest tests/test_nat_gpu.py tests/test_fw_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_natfw.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 tools/flows_sweep.py > $O/sweep_mask.log 2>&1 && \
VIGPATH_MIX=1 timeout -k 10 300 python3 tools/flows_sweep.py > $O/sweep_mix.log 2>&1 && \
timeout -k 10 300 python3 bench.py --no-cpu > $O/bench.log 2>&1
rc=$?
tail -3 $O/pytest_natfw.log; tail -2 $O/pytest_gpu.log; cat $O/sweep_mask.log $O/sweep_mix.log $O/bench.log
exit $rc
