set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_shard_gpu.py -q -x > gpurun_out/pytest_shard.log 2>&1 && \
VIGPATH_COMM=host timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --batch 4194304 --flows 1048576 > gpurun_out/bench_shard2.log 2>&1 && \
timeout -k 10 300 python3 bench.py > gpurun_out/bench.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_shard.log; tail -3 gpurun_out/bench_shard2.log; cat gpurun_out/bench.log
exit $rc
