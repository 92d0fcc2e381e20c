#!/bin/bash
# Kernel timeline of a medium host-buffer batch (AUTO, keyed all-comb) under rocprofv3 --kernel-trace.
# Run on the GPU box from the repo root:  tools/trace_medium.sh SIZE -> gpurun_out/medtrace_SIZE/
set -o pipefail
export TMPDIR=/tmp
N=${1:-10000}
OUT=gpurun_out/medtrace_$N
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace -o run -- python3 tools/latency_probe.py --sizes $N --reps 5 \
  --paths auto > $OUT/probe.json 2> $OUT/trace.log || exit $?
python3 tools/timeline.py $OUT/trace/run_results.db --steps 2 > $OUT/timeline.txt || exit $?
cat $OUT/timeline.txt
