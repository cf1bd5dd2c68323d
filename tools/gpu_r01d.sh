set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_shard_gpu.py -q -x > gpurun_out/pytest_shard.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_shard.log
exit $rc
