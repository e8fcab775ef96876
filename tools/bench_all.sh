#!/bin/bash
# One bench line per BASELINE.json config (c2 headline, c3 sweep, c4 wide,
# c5 sheet) on this box; stops at the first failure.
set -u
mkdir -p gpurun_out
for c in c2 c3 c4 c5; do
  case $c in
    c2) extra="--steps 5 --warmup 2";;
    c3) extra="--steps 3 --warmup 1 --profile-reps 1";;
    c4) extra="--steps 3 --warmup 1";;
    c5) extra="--steps 3 --warmup 1";;
  esac
  timeout -k 10 400 python bench.py --config $c $extra > gpurun_out/bench_$c.log 2>&1
  rc=$?
  echo "$c rc=$rc"; tail -1 gpurun_out/bench_$c.log
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/bench_$c.log; exit $rc; fi
done
