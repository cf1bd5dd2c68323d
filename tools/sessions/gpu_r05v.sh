#!/bin/bash
# round 5 session v: viglb -- backends staged with their header words (no
# dependent NIC-MAC load), one port per burst; tests, then config4_lb twice
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "lb or burst or shim" > gpurun_out/r05v_pytest.out 2>&1 || { tail -40 gpurun_out/r05v_pytest.out; exit 1; }
tail -1 gpurun_out/r05v_pytest.out
for i in 1 2; do
timeout -k 10 300 python3 tools/bench_extra.py config4_lb > gpurun_out/r05v_lb$i.out 2>&1 || { tail -20 gpurun_out/r05v_lb$i.out; exit 1; }
tail -1 gpurun_out/r05v_lb$i.out | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['config4_lb']; print(d['ms_per_step'], d['kernel_ms_per_launch'], d['frac'], d['parity']['match'], d['frac_basis'])"
done
