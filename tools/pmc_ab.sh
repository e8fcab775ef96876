#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes of one bench workload for several A/B
# libraries (each pass its own rocprofv3 run):
#   tools/pmc_ab.sh "lib1 lib2 ..." [bench args]  -> gpurun_out/pmcab_<lib>_{fetch,write}
set -u
export TMPDIR=/tmp
LIBS=$1; shift
for l in $LIBS; do
  for c in FETCH_SIZE WRITE_SIZE; do
    d=gpurun_out/pmcab_${l}_${c}
    mkdir -p $d
    YUMA_HIP_LIB=$PWD/ablib/$l.so timeout -s KILL 200 rocprofv3 --pmc $c --kernel-trace -T -f csv -d $d -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-also --profile-reps 1 "$@" > $d.log 2>&1
    rc=$?; echo "$l $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
