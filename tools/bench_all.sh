#!/bin/bash
# One bench line per BASELINE.json config (c2 headline, c3 sweep, c4 wide,
# c5 sheet) and the other c2 variants on this box; stops at the first failure.
#   tools/bench_all.sh [c2 c3 c4 c5 y1 y2 y0]...   (default: all)
set -u
mkdir -p gpurun_out
W=${*:-c2 c3 c4 c5 y1 y2 y0}
for c in $W; do
  case $c in
    c2) extra=(--steps 5 --warmup 2);;
    c3) extra=(--config c3 --steps 3 --warmup 1 --profile-reps 1);;
    c4) extra=(--config c4 --steps 3 --warmup 1);;
    c5) extra=(--config c5 --steps 3 --warmup 1);;
    y1) extra=(--version "Yuma 1 (paper)" --no-also --steps 5 --warmup 2);;
    y2) extra=(--version "Yuma 2 (Adrian-Fish)" --no-also --steps 5 --warmup 2);;
    y0) extra=(--version "Yuma 0 (subtensor)" --no-also --steps 5 --warmup 2);;
  esac
  timeout -k 10 400 python bench.py "${extra[@]}" > gpurun_out/bench_$c.log 2>&1
  rc=$?
  echo "$c rc=$rc"; tail -1 gpurun_out/bench_$c.log | cut -c1-400
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/bench_$c.log; exit $rc; fi
done
