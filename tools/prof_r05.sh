#!/bin/bash
# Round-5 profiles at HEAD (each rocprofv3 pass its own run; never --pmc with
# a trace domain): kernel trace + FETCH_SIZE / WRITE_SIZE passes per bench
# workload (tools/prof.sh), SQ passes (VALU / SALU issue, waits, clock) and
# the consensus kernels' LDS counters.
#   tools/prof_r05.sh [c2 c2y4l c3 c4 v1 v2 v0 sqc3 sqc4 sqc2 lds]...   (default: all)
set -u
export TMPDIR=/tmp
W=${*:-c2 c2y4l c3 c4 v1 v2 v0 sqc3 sqc4 sqc2 lds}
SQ="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
sq() {  # sq TAG [bench args]
  local tag=$1; shift
  mkdir -p gpurun_out/prof_$tag
  timeout -s KILL 150 rocprofv3 --pmc $SQ --kernel-trace -T -f csv -d gpurun_out/prof_$tag -o sq -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-also --profile-reps 1 "$@" > gpurun_out/prof_$tag/run.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
for w in $W; do
  case $w in
    c2) bash tools/prof.sh c2y3 || exit $? ;;
    c2y4l) bash tools/prof.sh c2y4l --version "Yuma 4 (Rhef+relative bonds) - liquid alpha on" || exit $? ;;
    c3) bash tools/prof.sh c3 --config c3 || exit $? ;;
    c4) bash tools/prof.sh c4 --config c4 || exit $? ;;
    v1) bash tools/prof.sh v1 --version "Yuma 1 (paper)" || exit $? ;;
    v2) bash tools/prof.sh v2 --version "Yuma 2 (Adrian-Fish)" || exit $? ;;
    v0) bash tools/prof.sh v0 --version "Yuma 0 (subtensor)" || exit $? ;;
    sqc3) sq sqc3 --config c3 ;;
    sqc4) sq sqc4 --config c4 ;;
    sqc2) sq sqc2 ;;
    lds) bash tools/prof_lds.sh || exit $? ;;
  esac
done
exit 0
