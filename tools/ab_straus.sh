#!/bin/bash
# A/B of engine builds on the Straus path (the bench batch forced per-request Straus), run on the GPU
# box from the repo root:  tools/ab_straus.sh ROUNDS name ...  ("base" = the product library, any other
# name = variants/<name>/libplenum_verify.so from tools/build_variant.sh)
set -o pipefail
ROUNDS=$1; shift
DS=/tmp/nym_ab.npz
[ -f $DS ] || timeout -k 10 300 python3 tools/nym_workload.py --out $DS > /dev/null || exit $?
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    if [ "$v" = base ]; then lib=""; else lib="PLENUM_AMD_LIB=variants/$v/libplenum_verify.so"; fi
    out=$(env $lib timeout -k 10 200 python3 bench.py --dataset $DS --no-cpu-baseline --no-config3 --sustain-s 0 \
          --no-host-path --no-ingress --no-multisig --steps 12 --warmup 2 2>/dev/null | tail -1) || exit $?
    echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['straus_path']; print('$v', d['ms_per_step'], d['stages_ms'], d['verdicts_ok'])"
  done
done
