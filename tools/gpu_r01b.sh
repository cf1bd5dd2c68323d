# GPU session: parity tests, NF side benches, mix-mode sweep, bench + profiles
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 tools/bench_nf.py > gpurun_out/bench_nf.log 2>&1 && \
VIGPATH_MIX=1 timeout -k 10 300 python3 tools/flows_sweep.py > gpurun_out/sweep_mix.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r01_kt -o kt -- python3 bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/r01_kt.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r01_fetch -o fetch -- python3 bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/r01_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r01_write -o write -- python3 bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/r01_write.log 2>&1
du -sh gpurun_out/* ; tail -3 gpurun_out/pytest_gpu.log
