#!/bin/bash
# round 4 session ap: the fold expands a run word with one lane's LDS atomic
# into a per-group maximum instead of 64 lanes' atomics: GPU suite, then the
# headline step against the previous commit's build (abtmp/), interleaved
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_session.sh r04ap tests || { tail -40 gpurun_out/r04ap_pytest.log; exit 1; }
grep -o "[0-9]* passed.*" gpurun_out/r04ap_pytest.log | tail -1
for v in old new old new old new; do
  d=.; [ $v = old ] && d=abtmp
  (cd $d && timeout -k 10 200 python3 bench.py --no-cpu --no-e2e --no-extra --steps 20) > gpurun_out/r04ap_$v.out 2>&1 || exit $?
  echo "$v $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_per_launch": [0-9.]*\|"match": [a-z]*' gpurun_out/r04ap_$v.out | tr '\n' ' ')"
done
rm -rf gpurun_out/r04ap_kt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04ap_kt -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-e2e --no-extra > gpurun_out/r04ap_kt.log 2>&1 || exit $?
echo done
