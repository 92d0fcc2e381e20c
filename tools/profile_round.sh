#!/bin/bash
# rocprofv3 evidence for the bench's kernels (run on the GPU box from the repo root):
#   1. --kernel-trace --stats of the bench command itself (per-kernel average durations)
#   2. separate --pmc passes (never combined with tracing options) for HBM bytes and VALU/occupancy
# Usage: tools/profile_round.sh TAG   -> gpurun_out/prof_TAG/...
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
DS=/tmp/nym_1m.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS || exit $?
BENCH="python3 bench.py --dataset $DS --no-cpu-baseline --no-host-path --no-config3 --sustain-s 0"
echo "== kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- $BENCH > $OUT/bench_traced.json 2> $OUT/trace.log || exit $?
PMCB="$BENCH --steps 3 --warmup 1"
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  echo "== pmc pass $i: $ctr"
  timeout -s KILL 240 rocprofv3 --pmc $ctr -d $OUT/pmc$i -o run -- $PMCB > $OUT/pmc$i.json 2> $OUT/pmc$i.log || exit $?
done
echo "== done"
