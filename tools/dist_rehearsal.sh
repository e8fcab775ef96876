#!/bin/bash
# Rehearsal of bench.py's N-rank path on a ONE-GPU box: N processes share the
# card, torch.distributed over gloo (YUMA_BENCH_BACKEND=gloo). The numbers are
# meaningless (ranks contend for one GPU); what is checked is that every config
# launches, shards, times, gathers and exits cleanly with one JSON line.
#   tools/dist_rehearsal.sh [N]   (default 2; results under gpurun_out/dist/)
set -o pipefail
N=${1:-2}
export TMPDIR=/tmp YUMA_BENCH_BACKEND=gloo
mkdir -p gpurun_out/dist
for cfg in c2 c3 c4 c5; do
  log=gpurun_out/dist/${cfg}_n${N}.log
  timeout -k 10 300 python -u bench.py --config $cfg --gpus $N --steps 2 --warmup 1 > $log 2>&1
  rc=$?
  echo "$cfg n$N rc=$rc"
  tail -1 $log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(' ', d['n_gpus'], d['value'], d['ms_per_step'], d['config'].get('parallelism'), 'cpu_baseline' in d)" || tail -20 $log
  [ $rc -eq 0 ] || exit $rc
done
