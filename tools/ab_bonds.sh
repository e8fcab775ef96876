# Phase times of the c2 bond-scan workloads (Yuma 3 with history, Yuma 4
# liquid with history, Yuma 3 without history) for the library in
# YUMA_HIP_LIB (default: the in-tree build) — the A/B harness behind the
# bond-kernel choices in DESIGN.md section 2.
export TMPDIR=/tmp
for v in y3 y4l y3nh; do
  case $v in
    y3) A=(--version "Yuma 3 (Rhef)");;
    y4l) A=(--version "Yuma 4 (Rhef+relative bonds)" --liquid);;
    y3nh) A=(--version "Yuma 3 (Rhef)" --no-history);;
  esac
  timeout -k 10 120 python -u tools/phase_times.py "${A[@]}" --tag "$v ${TAG:-}" >> gpurun_out/ab_bonds.txt 2>&1 || exit 1
done
