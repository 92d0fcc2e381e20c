#!/bin/bash
# A/B of engine builds on the bench workload (run on the GPU box from the repo root):
#   microbench/ab_bench.sh ROUNDS lib1 lib2 ...   (libs under microbench/variants/, without .so)
# One synthetic NYM dataset (tools/nym_workload.py), then ROUNDS interleaved passes of
# bench.py --dataset per build; prints each run's stage times.
set -o pipefail
ROUNDS=$1; shift
DS=/tmp/nym_ab.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > /dev/null || exit $?
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    out=$(PLENUM_AMD_LIB=microbench/variants/$v.so timeout -k 10 200 python3 bench.py --dataset $DS --no-cpu-baseline \
          --no-host-path --no-ingress --no-config3 --no-multisig ${AB_EXTRA:-} --steps 30 --warmup 3 2>/dev/null | tail -1) || exit $?
    echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['pipeline']; s=d.get('straus_path',{}); print('$v', d['ms_per_step'], {k: p[k] for k in ('keys_ms','prep_ms','table_ms','msm_ms','encode_ms')}, d['verdicts_ok'], 'straus', s.get('ms_per_step'), s.get('stages_ms'), s.get('verdicts_ok'))"
  done
done
