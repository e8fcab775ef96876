#!/bin/bash
# A/B on the c4 shape (256 x 65536 x 100, no history): Yuma 4 liquid and Yuma 3
# per-phase device time, per library, two rounds.
export TMPDIR=/tmp
for rep in 1 2; do
  for l in "$@"; do
    t=$(basename $l .so)
    YUMA_HIP_LIB=$PWD/$l timeout -k 10 120 python -u tools/phase_times.py --no-history --M 65536 --epochs 100 --version "Yuma 4 (Rhef+relative bonds)" --liquid --tag "$t c4 y4l" || exit 1
    YUMA_HIP_LIB=$PWD/$l timeout -k 10 120 python -u tools/phase_times.py --no-history --M 65536 --epochs 100 --tag "$t c4 y3" || exit 1
  done
done
