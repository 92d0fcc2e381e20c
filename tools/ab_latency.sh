#!/bin/bash
# A/B of library variants on small host-buffer calls (1 and 100 requests, median of 300 calls each,
# tools/lat_breakdown.py run; no tracing). Usage on the GPU box: tools/ab_latency.sh VARIANT... ("base" =
# the in-tree library)
set -o pipefail
mkdir -p gpurun_out/ablat
for round in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then unset PLENUM_AMD_LIB; else export PLENUM_AMD_LIB=variants/$v/libplenum_verify.so; fi
    timeout -k 10 120 python3 tools/lat_breakdown.py run 300 ${SIZES:-1,100} > gpurun_out/ablat/$v.$round.json 2> gpurun_out/ablat/$v.$round.log || exit $?
    echo "$v $(cat gpurun_out/ablat/$v.$round.json)"
  done
done
