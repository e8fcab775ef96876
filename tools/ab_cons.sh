#!/bin/bash
# A/B of consensus kernels (ablib/*.so from tools/ab_build.py): per-phase
# device time of the c2 Yuma 3 workload, two rounds.
export TMPDIR=/tmp
for rep in 1 2; do
  for l in "$@"; do
    YUMA_HIP_LIB=$PWD/$l timeout -k 10 120 python -u tools/phase_times.py --tag "$(basename $l .so)" || exit 1
  done
done
