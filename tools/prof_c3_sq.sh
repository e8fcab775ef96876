#!/bin/bash
# c3 sweep step counters: one SQ pass (VALU issue, waits) and one L2 hit/miss
# pass, each its own rocprofv3 run (gpurun_out/prof_c3sq, gpurun_out/prof_c3tcc).
set -u
export TMPDIR=/tmp
C="${SQC:-SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM}"
mkdir -p gpurun_out/prof_c3sq gpurun_out/prof_c3tcc
timeout -s KILL 150 rocprofv3 --pmc $C --kernel-trace -T -f csv -d gpurun_out/prof_c3sq -o sq -- python3 bench.py --config c3 --steps 1 --warmup 1 --no-cpu-baseline --profile-reps 1 > gpurun_out/prof_c3sq/run.log 2>&1
rc=$?; echo "sq rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -T -f csv -d gpurun_out/prof_c3tcc -o tcc -- python3 bench.py --config c3 --steps 1 --warmup 1 --no-cpu-baseline --profile-reps 1 > gpurun_out/prof_c3tcc/run.log 2>&1
rc=$?; echo "tcc rc=$rc"; exit $rc
