#!/bin/bash
# Kernel timeline of the bench's configs[2] leg (2 % adversarial, AUTO split into comb keys and a
# Straus side stream) and of the headline for comparison. Run on the GPU box from the repo root:
#   tools/trace_config3.sh [TAG]  -> gpurun_out/c3trace[_TAG]/{timeline_headline,timeline_config3,steps}.txt
# (PLENUM_AMD_LIB selects a variant library as everywhere else)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/c3trace${1:+_$1}
mkdir -p $OUT
DS=/tmp/nym_c3.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > /dev/null || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace -o run -- python3 bench.py --dataset $DS --no-cpu-baseline \
  --no-host-path --no-ingress --no-multisig --no-straus --steps 4 --warmup 1 > $OUT/bench.json 2> $OUT/trace.log || exit $?
DB=$(ls $OUT/trace/*/run_results.db $OUT/trace/*.db $OUT/trace/*/*.db 2>/dev/null | head -1)
echo "db: $DB"
# the config3 leg runs after the headline: its steps are the last ones in the trace
python3 tools/timeline.py "$DB" --steps 2 > $OUT/timeline_config3.txt || exit $?
python3 tools/timeline.py "$DB" --steps 9 | head -60 > $OUT/timeline_headline.txt || true
python3 tools/timeline.py "$DB" --summary > $OUT/steps.txt || exit $?
cat $OUT/steps.txt
