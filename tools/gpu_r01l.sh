# Round-1 GPU session l: ablation incl. contiguous per-block tile ranges.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python3 tools/ablate.py 5 > $O/ablate.log 2>&1
rc=$?
cat $O/ablate.log
exit $rc
