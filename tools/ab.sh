#!/bin/bash
# A/B: fused phase 1 vs multi-pass (YUMA_NO_FUSED=1), one bench line each
set -u
mkdir -p gpurun_out
for mode in fused unfused; do
  if [ $mode = unfused ]; then export YUMA_NO_FUSED=1; else unset YUMA_NO_FUSED; fi
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/ab_$mode.log 2>&1
  rc=$?
  echo "$mode rc=$rc"; tail -1 gpurun_out/ab_$mode.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], {k:v['ms'] for k,v in d['phases'].items() if v['ms']>0})" 2>/dev/null || tail -3 gpurun_out/ab_$mode.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
