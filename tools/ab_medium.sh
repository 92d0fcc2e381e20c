#!/bin/bash
# A/B of engine builds at medium batch sizes (host-buffer calls, AUTO), interleaved on one box:
#   tools/ab_medium.sh ROUNDS SIZES lib1 lib2 ...   (libs under microbench/variants/, without .so)
set -o pipefail
ROUNDS=$1; SIZES=$2; shift 2
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    out=$(PLENUM_AMD_LIB=microbench/variants/$v.so timeout -k 10 200 python3 tools/latency_probe.py --sizes $SIZES \
          --reps 15 --paths auto 2>/dev/null | tail -1) || exit $?
    echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['results']['auto']; print('$v', {k: (v['median_ms'], v['device_ms'], v['ok']) for k, v in d.items()})"
  done
done
