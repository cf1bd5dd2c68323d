#!/bin/bash
# round 4 session aq: the lean tile writes its out-port through (sc1) so the
# port array is not left dirty in the L2s at the kernel end: GPU suite, then
# the headline step against the previous commit's build (abtmp/), interleaved.
# Slower (kernel +3.5 us, step +5 us; the boundary unchanged): not kept
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_session.sh r04aq test:nat || { tail -40 gpurun_out/r04aq_pytest_nat.log; exit 1; }
grep -o "[0-9]* passed.*" gpurun_out/r04aq_pytest_nat.log | tail -1
for v in old new old new old new; do
  d=.; [ $v = old ] && d=abtmp
  (cd $d && timeout -k 10 200 python3 bench.py --no-cpu --no-e2e --no-extra --steps 20) > gpurun_out/r04aq_$v.out 2>&1 || exit $?
  echo "$v $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*' gpurun_out/r04aq_$v.out | tr '\n' ' ')"
done
rm -rf gpurun_out/r04aq_kt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04aq_kt -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-e2e --no-extra > gpurun_out/r04aq_kt.log 2>&1 || exit $?
echo done
