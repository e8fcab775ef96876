#!/bin/bash
# chunk-size sweep of bench.py (no CPU baseline); one JSON line per setting
set -u
mkdir -p gpurun_out
for c in "$@"; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --chunk $c > gpurun_out/sweep_c$c.log 2>&1
  rc=$?
  echo "chunk=$c rc=$rc"; tail -1 gpurun_out/sweep_c$c.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], {k:v['ms'] for k,v in d['phases'].items()})" 2>/dev/null
  if [ $rc -ne 0 ]; then exit $rc; fi
done
