#!/bin/bash
# rocprofv3 passes for the bench workload: kernel trace + stats, then two
# separate PMC passes (FETCH_SIZE / WRITE_SIZE) and one SQ pass.
set -u
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --profile-reps 1"
run() { local name=$1; shift; echo "== $name"; timeout -k 10 600 "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -2 $OUT/$name.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
run trace rocprofv3 --kernel-trace --stats -T -f csv -d $OUT/prof_trace -o run -- $B
run pmc_fetch rocprofv3 --pmc FETCH_SIZE --kernel-trace -T -f csv -d $OUT/pmc_fetch -o fetch -- $B
run pmc_write rocprofv3 --pmc WRITE_SIZE --kernel-trace -T -f csv -d $OUT/pmc_write -o write -- $B
run pmc_sq rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES --kernel-trace -T -f csv -d $OUT/pmc_sq -o sq -- $B
exit 0
