#!/bin/bash
# A/B per-phase device time on c2 (Yuma 3 with history) and c4 (Yuma 3 no
# history, 256 x 65536 x 100), per library, two rounds.
export TMPDIR=/tmp
for rep in 1 2; do
  for l in "$@"; do
    t=$(basename $l .so)
    YUMA_HIP_LIB=$PWD/$l timeout -k 10 120 python -u tools/phase_times.py --tag "$t c2" || exit 1
    YUMA_HIP_LIB=$PWD/$l timeout -k 10 120 python -u tools/phase_times.py --no-history --M 65536 --epochs 100 --tag "$t c4" || exit 1
  done
done
