#!/bin/bash
# LDS counters for k_consensus_p with two libraries (c2 200 epochs)
set -u
export TMPDIR=/tmp
C="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for l in ${LDSLIBS:-base cp_swz}; do
  mkdir -p gpurun_out/lds_$l
  YUMA_HIP_LIB=$PWD/ablib/$l.so timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -T -f csv -d gpurun_out/lds_$l -o lds -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-also --profile-reps 1 --epochs 200 > gpurun_out/lds_$l/run.log 2>&1
  rc=$?; echo "$l rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
