#!/bin/bash
# Run GPU steps in order; each "name|seconds|command" line runs under its own timeout.  A step
# that fails with a plain test failure (exit 1) lets the next one run; a fault, abort, segfault,
# timeout or any other status ends the script (no further GPU work in this call).
set -u
mkdir -p gpurun_out
while IFS= read -r line; do
  [ -z "$line" ] && continue
  name="${line%%|*}"; rest="${line#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== $name ($secs s): $cmd" | tee -a gpurun_out/steps.log
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done
