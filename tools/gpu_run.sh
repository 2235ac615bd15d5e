#!/bin/bash
# Runs GPU test files one after another; stops at the first crash/timeout (exit code not 0/1).
mkdir -p gpurun_out
for f in "$@"; do
  name=$(basename "$f" .py)
  timeout -k 10 900 python -u -m pytest "$f" -q -m gpu -rf -p no:cacheprovider --tb=short --timeout 300 --timeout-method thread -s > gpurun_out/$name.log 2>&1
  rc=$?
  echo "$f rc=$rc"; tail -5 gpurun_out/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: crash or timeout in $f"; exit $rc; fi
done
exit 0
