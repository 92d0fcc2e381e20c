#!/bin/bash
# Run GPU steps in order; stop at the first step that faults, aborts or times out
# (exit codes other than 0 = ok / 1 = ordinary test failure). Usage:
#   tools/gpu_steps.sh "name1:::timeout1:::cmd1" "name2:::timeout2:::cmd2" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:::*}"; rest="${spec#*:::}"; to="${rest%%:::*}"; cmd="${rest#*:::}"
  echo "=== step $name (timeout ${to}s): $cmd"
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== step $name rc=$rc"
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "=== stopping after $name (rc=$rc)"; exit $rc; fi
done
exit 0
