#!/bin/bash
# LDS counters of the consensus (weighted-median) kernels (north_star: "LDS
# bank-conflict counters for the median kernel"): the wave-owned
# k_consensus_w (V <= 256, the bench path: DPP reductions, no LDS) and the
# LDS-reducing k_consensus (V > 256).
set -u
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
C="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
run() { local name=$1; shift; echo "== $name"; timeout -s KILL 120 "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -1 $OUT/$name.log | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }
run pmc_lds_v256 rocprofv3 --pmc $C --kernel-trace -T -f csv -d $OUT/pmc_lds_v256 -o lds -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --profile-reps 1 --epochs 200
run pmc_lds_v512 rocprofv3 --pmc $C --kernel-trace -T -f csv -d $OUT/pmc_lds_v512 -o lds -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --profile-reps 1 --epochs 100 --validators 512
exit 0
