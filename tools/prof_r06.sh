#!/bin/bash
# Round-6 profiles, all from ONE library build (bench.py prints its
# engine_build_id in every line; tools/pmc_traffic.py and tools/sq_summary.py
# record it, and bench.py pairs a counter record only with runs of the same
# build). Each rocprofv3 pass is its own run (never --pmc with a trace domain):
# kernel trace + FETCH_SIZE / WRITE_SIZE passes per bench workload
# (tools/prof.sh), SQ passes (VALU / SALU issue, waits, clock), and the LDS
# pass of the consensus kernel at c2 and c4.
#   tools/prof_r06.sh [c2 c2y4l c3 c4 v1 v2 v0 sqc2 sqc3 sqc4 sqv0 ldsc2 ldsc4]...   (default: all)
set -u
export TMPDIR=/tmp
W=${*:-c2 c2y4l c3 c4 v1 v2 v0 sqc2 sqc3 sqc4 sqv0 ldsc2 ldsc4}
SQ="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
LDS="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
pass() {  # pass TAG COUNTERS [bench args]
  local tag=$1 ctr=$2; shift 2
  mkdir -p gpurun_out/prof_$tag
  timeout -s KILL 200 rocprofv3 --pmc $ctr --kernel-trace -T -f csv -d gpurun_out/prof_$tag -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-also --profile-reps 1 "$@" > gpurun_out/prof_$tag/run.log 2>&1
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
    sqc2) pass sqc2 "$SQ" ;;
    sqc3) pass sqc3 "$SQ" --config c3 ;;
    sqc4) pass sqc4 "$SQ" --config c4 ;;
    sqv0) pass sqv0 "$SQ" --version "Yuma 0 (subtensor)" ;;
    ldsc2) pass ldsc2 "$LDS" ;;
    ldsc4) pass ldsc4 "$LDS" --config c4 ;;
  esac
done
exit 0
