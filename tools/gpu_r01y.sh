# Round-1 GPU session y: vigpol parity, then the whole GPU suite and smoke.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_pol_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest_pol.log 2>&1
rc=$?
tail -15 $O/pytest_pol.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -5 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?
tail -3 $O/smoke.log
exit $rc
