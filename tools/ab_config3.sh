#!/bin/bash
# A/B of library variants on the headline and the configs[2] (2 % adversarial) leg.
# Usage on the GPU box from the repo root: tools/ab_config3.sh VARIANT... ("base" = the in-tree library)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/ab
mkdir -p $OUT
DS=/tmp/nym_ab.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > /dev/null || exit $?
for round in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then unset PLENUM_AMD_LIB; else export PLENUM_AMD_LIB=variants/$v/libplenum_verify.so; fi
    timeout -k 10 300 python3 bench.py --dataset $DS --no-cpu-baseline --no-host-path \
      --no-ingress --no-multisig --no-straus --steps 20 --warmup 5 > $OUT/$v.$round.json 2> $OUT/$v.$round.log || exit $?
    python3 - "$v" "$OUT/$v.$round.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
c3 = d.get("config3") or {}
print(sys.argv[1], "headline", round(d["value"] / 1e6, 1), "M/s", d["ms_per_step"], "ms | config3",
      round(c3.get("value", 0) / 1e6, 1), "M/s", c3.get("ms_per_step"), "ms")
PY
  done
done
