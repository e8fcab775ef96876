#!/bin/bash
# A/B of engine builds on the c3 sweep step (bench.py --config c3), two rounds.
export TMPDIR=/tmp
for rep in 1 2; do
  for l in "$@"; do
    t=$(basename $l .so)
    YUMA_HIP_LIB=$PWD/$l timeout -k 10 200 python -u bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline --profile-reps 1 > gpurun_out/c3_$t.log 2>&1 || exit 1
    tail -1 gpurun_out/c3_$t.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('$t c3', d['value'], d['ms_per_step'], {k:v['ms'] for k,v in d['phases'].items()})"
  done
done
