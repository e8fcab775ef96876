#!/bin/bash
# A/B an engine env knob: tools/ab.sh VAR val1 val2 ... [-- extra bench.py args]
# One bench line per setting ("-" = unset), printed as value, ms/step, phase ms.
set -u
mkdir -p gpurun_out
var=$1; shift
vals=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do vals+=("$1"); shift; done
[ $# -gt 0 ] && shift
for v in "${vals[@]}"; do
  if [ "$v" = "-" ]; then unset "$var"; else export "$var=$v"; fi
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --profile-reps 2 "$@" > gpurun_out/ab_${var}_${v}.log 2>&1
  rc=$?
  echo "$var=$v rc=$rc"; tail -1 gpurun_out/ab_${var}_${v}.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], {k:v['ms'] for k,v in d['phases'].items() if v['ms']>0})" 2>/dev/null || tail -3 gpurun_out/ab_${var}_${v}.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
