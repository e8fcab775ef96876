#!/bin/bash
# rocprofv3 passes over one bench workload, each its own run (never --pmc
# together with a trace domain): kernel trace + stats, then FETCH_SIZE and
# WRITE_SIZE in separate passes (MI355X_MICROARCH.md, HBM section).
#   tools/prof.sh TAG [bench.py args...]   -> gpurun_out/prof_TAG/{trace,fetch,write}
# Afterwards (on the CPU side): tools/pmc_traffic.py gpurun_out/prof_TAG/fetch gpurun_out/prof_TAG/write ...
set -u
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
B=(python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-also --profile-reps 1 "$@")
run() {
  local name=$1; shift
  echo "== $TAG $name"
  timeout -k 10 300 "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "rc=$rc"; tail -1 $OUT/$name.log | cut -c1-300
  if [ $rc -ne 0 ]; then tail -20 $OUT/$name.log; exit $rc; fi
}
run trace rocprofv3 --kernel-trace --stats -T -f csv -d $OUT/trace -o run -- "${B[@]}"
run fetch rocprofv3 --pmc FETCH_SIZE --kernel-trace -T -f csv -d $OUT/fetch -o fetch -- "${B[@]}"
run write rocprofv3 --pmc WRITE_SIZE --kernel-trace -T -f csv -d $OUT/write -o write -- "${B[@]}"
exit 0
