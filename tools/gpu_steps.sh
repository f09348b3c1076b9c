#!/bin/bash
# Run named GPU steps in order, each under its own time limit; stop at the first step
# that crashes, aborts, faults or times out (exit >= 124).  Ordinary failures (exit 1,
# e.g. a failing assertion) are recorded and the next step still runs.
# usage: tools/gpu_steps.sh "name|seconds|command" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
status=0
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] exit $rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then status=$rc; fi
  if [ $rc -ge 124 ]; then echo "stopping: step $name ended with $rc"; exit $rc; fi
done
exit $status
