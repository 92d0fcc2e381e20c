#!/bin/bash
# Build engine variants (compile-time switches of csrc/pv_engine.hip) next to each other for A/B
# timing on the GPU:
#   microbench/build_variants.sh NAME "-DFLAG=.. ..." [NAME "FLAGS" ...]  -> microbench/variants/NAME.so
# Only the engine is recompiled with the flags; the other objects come from the in-tree build
# (make -C indy-plenum_amd first). Load one with PLENUM_AMD_LIB=microbench/variants/NAME.so
# (tests/perf_quick.py, bench.py).
cd "$(dirname "$0")/../indy-plenum_amd" || exit 1
mkdir -p ../microbench/variants
OTHERS="build/pv_latency.hip.o build/pv_ingress.hip.o build/host_prep.cpp.o build/signing_json.cpp.o"
for o in $OTHERS; do [ -f "$o" ] || { echo "missing $o: run make -C indy-plenum_amd" >&2; exit 1; }; done
pids=()
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  V=../microbench/variants/$name
  ( /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -Wall $flags -c -o $V.engine.o csrc/pv_engine.hip &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -fPIC -shared -o $V.so $V.engine.o $OTHERS \
      -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib && rm -f $V.engine.o ) > $V.build.txt 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=1; done
exit $rc
