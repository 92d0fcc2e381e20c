#!/bin/bash
# A/B of run-time knobs on the headline and configs[2] legs (GPU box, repo root):
#   tools/ab_env.sh ROUNDS "name:VAR=val VAR2=val" "base:" ...   -> gpurun_out/ab_env/<name>.<round>.json
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/ab_env
mkdir -p $OUT
ROUNDS=$1; shift
DS=/tmp/nym_ab.npz
[ -f $DS ] || timeout -k 10 300 python3 tools/nym_workload.py --out $DS > /dev/null || exit $?
for round in $(seq 1 $ROUNDS); do
  for spec in "$@"; do
    name="${spec%%:*}"; envs="${spec#*:}"
    env $envs timeout -k 10 300 python3 bench.py --dataset $DS --no-cpu-baseline --no-host-path \
      --no-ingress --no-multisig --no-straus ${AB_EXTRA:-} --steps 20 --warmup 5 > $OUT/$name.$round.json 2> $OUT/$name.$round.log || exit $?
    python3 - "$name" "$OUT/$name.$round.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
c3 = d.get("config3") or {}
p = d["pipeline"]
print(sys.argv[1], "headline", round(d["value"] / 1e6, 1), "M/s", d["ms_per_step"], "ms", {k: p[k] for k in ("keys_ms", "prep_ms", "table_ms", "msm_ms", "encode_ms")}, d["verdicts_ok"],
      "| config3", round(c3.get("value", 0) / 1e6, 1), "M/s", c3.get("ms_per_step"), "ms", c3.get("verdicts_match_libsodium"))
PY
  done
done
