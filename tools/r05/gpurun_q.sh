#!/bin/bash
# Submit one gpurun call, waiting while the pool reports no free box/slot
# (exit 3: nothing ran, nothing charged); any other outcome is returned as is.
# usage: tools/r05/gpurun_q.sh <timeout_s> <out_file> <command>
T=$1; OUT=$2; shift 2
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > "$OUT" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$OUT"; then exit $rc; fi
  sleep 90
done
exit $rc
