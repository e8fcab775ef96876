#!/bin/bash
# A/B of bond-scan shapes (ablib/*.so from tools/ab_build.py): per-phase
# device time of the c2 workloads with the bond history (Yuma 3, Yuma 4
# liquid), two rounds so box drift shows.
export TMPDIR=/tmp
for rep in 1 2; do
  for l in "$@"; do
    for v in y3 y4l; do
      case $v in
        y3) A=(--version "Yuma 3 (Rhef)");;
        y4l) A=(--version "Yuma 4 (Rhef+relative bonds)" --liquid);;
      esac
      YUMA_HIP_LIB=$PWD/$l timeout -k 10 120 python -u tools/phase_times.py "${A[@]}" --tag "$(basename $l .so) $v" || exit 1
    done
  done
done
