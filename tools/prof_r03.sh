#!/bin/bash
# Round-3 profiles at HEAD: kernel trace + FETCH/WRITE passes (tools/prof.sh)
# for the c2 line (Yuma 3) and its Yuma 4 liquid companion, the c3 sweep and
# the c4 wide subnet; then one SQ pass over the c2 step.
#   tools/prof_r03.sh [c2|c3|c4|sq]...   (default: all)
set -u
export TMPDIR=/tmp
W=${*:-c2 c3 c4 sq}
for w in $W; do
  case $w in
    c2) bash tools/prof.sh c2y3 || exit $?
        bash tools/prof.sh c2y4l --version "Yuma 4 (Rhef+relative bonds) - liquid alpha on" || exit $? ;;
    c3) bash tools/prof.sh c3 --config c3 || exit $? ;;
    c4) bash tools/prof.sh c4 --config c4 || exit $? ;;
    sq) C="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM"
        mkdir -p gpurun_out/prof_sq
        timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -T -f csv -d gpurun_out/prof_sq -o sq -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-also --profile-reps 1 > gpurun_out/prof_sq/run.log 2>&1
        echo "sq rc=$?" ;;
  esac
done
exit 0
