#!/bin/bash
# A/B engine knobs in one GPU call: tools/ab_env.sh "VAR=a" "VAR=b" ... [-- bench args]
# One bench line per setting: value, ms/step, per-phase ms.
set -u
mkdir -p gpurun_out
cfgs=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do cfgs+=("$1"); shift; done
[ $# -gt 0 ] && shift
for cfg in "${cfgs[@]}"; do
  env $cfg timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > "gpurun_out/ab_$cfg.log" 2>&1 || exit $?
  echo "$cfg $(tail -1 "gpurun_out/ab_$cfg.log" | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], {k:v['ms'] for k,v in d['phases'].items() if v['ms']>0})")"
done
