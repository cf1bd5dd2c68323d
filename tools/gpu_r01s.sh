# Round-1 GPU session s: table-size sweep, masked-CRC vs multiplicative home buckets.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
export SWEEP_FLOWS=1048576,4194304,8388608,16777216
timeout -k 10 300 python3 tools/flows_sweep.py > $O/sweep_mask.log 2>&1 && \
VIGPATH_MIX=1 timeout -k 10 300 python3 tools/flows_sweep.py > $O/sweep_mix.log 2>&1
rc=$?
cat $O/sweep_mask.log $O/sweep_mix.log
exit $rc
