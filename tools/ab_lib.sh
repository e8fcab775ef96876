#!/bin/bash
# A/B engine builds: tools/ab_lib.sh lib1.so lib2.so ... [-- extra bench.py args]
# One bench line per library (YUMA_HIP_LIB), printed as value, ms/step, phase ms.
set -u
mkdir -p gpurun_out
libs=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do libs+=("$1"); shift; done
[ $# -gt 0 ] && shift
for rep in 1 2; do
for l in "${libs[@]}"; do
  tag=$(basename "$l" .so)
  YUMA_HIP_LIB=$PWD/$l timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --profile-reps 2 "$@" > gpurun_out/ablib_${tag}.log 2>&1
  rc=$?
  echo "$tag rc=$rc"; tail -1 gpurun_out/ablib_${tag}.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], {k:v['ms'] for k,v in d['phases'].items() if v['ms']>0})" 2>/dev/null || tail -3 gpurun_out/ablib_${tag}.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
done
