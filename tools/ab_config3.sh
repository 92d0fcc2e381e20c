#!/bin/bash
# A/B of engine builds on the configs[2] leg (2 % adversarial records: AUTO splits the chunk into comb
# keys and a few thousand Straus requests on a side stream). Run on the GPU box from the repo root:
#   tools/ab_config3.sh ROUNDS lib1 lib2 ...   (libs under microbench/variants/, without .so)
set -o pipefail
ROUNDS=$1; shift
DS=/tmp/nym_ab.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > /dev/null || exit $?
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    out=$(PLENUM_AMD_LIB=microbench/variants/$v.so timeout -k 10 200 python3 bench.py --dataset $DS --no-cpu-baseline \
          --no-host-path --no-ingress --no-multisig --no-straus --steps 20 --warmup 3 2>/dev/null | tail -1) || exit $?
    echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config3']; print('$v', 'headline', d['ms_per_step'], d['verdicts_ok'], 'config3', c['ms_per_step'], c['stages_ms'], c['split'])"
  done
done
