#!/usr/bin/env bash
# Run GPU steps in order, each under its own timeout; a crash-class exit (timeout 124/137,
# abort 134, segfault 139, or any signal) ends the session, ordinary failures (exit 1) don't.
# usage: tools/gpu_steps.sh "name|seconds|command" ...
set -u
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] (${secs}s) $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] exit $rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "=== stopping: crash-class exit from [$name]"
    exit $rc
  fi
done
