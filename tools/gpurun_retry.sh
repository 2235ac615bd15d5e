#!/bin/bash
# retry a gpurun call while the pool reports no free slot/box (exit 3: nothing ran, nothing charged)
# usage: tools/gpurun_retry.sh OUTFILE TIMEOUT 'command'
out=$1; to=$2; shift 2
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$out" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$out"; then exit $rc; fi
  sleep 60
done
exit 3
