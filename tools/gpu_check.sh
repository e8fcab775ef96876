#!/bin/bash
# GPU-box check sequence: smoke, parity tests, bench, rocprofv3 kernel trace,
# per-phase times of the column-normalised variants. Each GPU step has its own
# time limit; a fault/abort/timeout stops the script (no further GPU work), a
# plain test failure (exit 1) does not.
#   tools/gpu_check.sh [smoke,tests,bench,prof,variants]   (default: all)
set -u
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
stage() {  # stage <name> <timeout-s> <cmd...>
  local name=$1 lim=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/stages.log
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/stages.log
  tail -5 $OUT/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
WHAT=${1:-all}
if [[ $WHAT == all || $WHAT == *smoke* ]]; then stage smoke 600 python -c "import __graft_entry__ as g; g.smoke()"; fi
if [[ $WHAT == all || $WHAT == *tests* ]]; then
  stage pytest_gpu 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
fi
if [[ $WHAT == all || $WHAT == *bench* ]]; then stage bench 900 python bench.py --steps 5 --warmup 2; fi
if [[ $WHAT == all || $WHAT == *prof* ]]; then
  stage rocprof 900 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --profile-reps 1
fi
if [[ $WHAT == all || $WHAT == *variants* ]]; then
  for v in "Yuma 1 (paper)" "Yuma 2 (Adrian-Fish)" "Yuma 0 (subtensor)"; do
    stage "phases_${v:5:1}" 300 python -u tools/phase_times.py --version "$v" --reps 2
  done
fi
exit 0
