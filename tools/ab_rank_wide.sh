#!/bin/bash
# A/B of the wide rank (k_rank_sw): c4 (history-less, 256 x 65536 x 100) and
# Yuma 1 at c2's shape (the bond-column-sum rank), per library, two rounds.
#   tools/ab_rank_wide.sh lib1.so lib2.so ...
export TMPDIR=/tmp
for rep in 1 2; do
  for l in "$@"; do
    t=$(basename $l .so)
    YUMA_HIP_LIB=$PWD/$l timeout -k 10 120 python -u tools/phase_times.py --no-history --M 65536 --epochs 100 --tag "$t c4" || exit 1
    YUMA_HIP_LIB=$PWD/$l timeout -k 10 120 python -u tools/phase_times.py --version "Yuma 1 (paper)" --tag "$t y1" || exit 1
  done
done
