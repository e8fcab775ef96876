#!/bin/bash
# gpurun with a wait-and-retry while the pool has no free slot or box (those
# calls run nothing and charge nothing); any call that ran returns as is.
#   tools/gpurun_retry.sh TIMEOUT 'command' [tries]
t=$1; cmd=$2; tries=${3:-15}
for i in $(seq 1 "$tries"); do
  out=$(/usr/local/graft/bin/gpurun --timeout "$t" -- "$cmd" 2>&1); rc=$?
  if echo "$out" | grep -q "nothing was charged\|no free box right now\|backing off"; then
    echo "[retry $i] pool busy; waiting" >&2; sleep 150; continue
  fi
  echo "$out"; exit $rc
done
echo "pool busy after $tries tries" >&2; exit 3
