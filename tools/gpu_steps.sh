#!/bin/bash
# Run named GPU steps, each under its own time limit; stop at the first step
# that faults, aborts or times out (rc other than 0/1), as gpurun requires.
#   tools/gpu_steps.sh "name|limit_s|command" ...   -> gpurun_out/<name>.log
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; lim=${rest%%|*}; cmd=${rest#*|}
  echo "== $name ($lim s): $cmd" | tee -a gpurun_out/steps.log
  timeout -k 10 "$lim" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done
exit 0
