#!/bin/bash
# Round-2 profiles at HEAD: kernel trace + FETCH/WRITE passes for the c2
# Yuma 3 line and its Yuma 4 liquid companion (tools/prof.sh), then one SQ
# counter pass over the c2 Yuma 3 step (instruction mix / waits per kernel).
set -u
export TMPDIR=/tmp
bash tools/prof.sh c2y3 || exit $?
bash tools/prof.sh c2y4l --version "Yuma 4 (Rhef+relative bonds) - liquid alpha on" || exit $?
C="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM"
mkdir -p gpurun_out/prof_sq
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -T -f csv -d gpurun_out/prof_sq -o sq -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-also --profile-reps 1 > gpurun_out/prof_sq/run.log 2>&1
echo "sq rc=$?"
