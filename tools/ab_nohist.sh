#!/bin/bash
# A/B of bond-scan shapes without the bond history: c2 (Yuma 3, no history),
# c4 (256 x 65536 x 100, Yuma 3) and the c3 sweep step, for each library.
export TMPDIR=/tmp
for rep in 1 2; do
  for l in "$@"; do
    t=$(basename $l .so)
    YUMA_HIP_LIB=$PWD/$l timeout -k 10 120 python -u tools/phase_times.py --no-history --tag "$t c2nh" || exit 1
    YUMA_HIP_LIB=$PWD/$l timeout -k 10 120 python -u tools/phase_times.py --no-history --M 65536 --epochs 100 --tag "$t c4" || exit 1
    YUMA_HIP_LIB=$PWD/$l timeout -k 10 200 python -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --profile-reps 1 > gpurun_out/c3_$t.log 2>&1 || exit 1
    tail -1 gpurun_out/c3_$t.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('$t c3', d['value'], d['ms_per_step'], {k:v['ms'] for k,v in d['phases'].items()})"
  done
done
