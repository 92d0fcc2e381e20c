#!/bin/bash
# Build engine variants (compile-time switches) next to each other for A/B timing on the GPU:
#   microbench/build_variants.sh NAME "-DFLAG=.. ..." [NAME "FLAGS" ...]  -> microbench/variants/NAME.so
# Load one with PLENUM_AMD_LIB=microbench/variants/NAME.so (tests/perf_quick.py, bench.py).
cd "$(dirname "$0")/../indy-plenum_amd" || exit 1
SRC="csrc/pv_engine.hip csrc/pv_latency.hip csrc/pv_ingress.hip csrc/host_prep.cpp csrc/signing_json.cpp"
pids=()
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared $flags -o ../microbench/variants/$name.so $SRC \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib > ../microbench/variants/$name.build.txt 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=1; done
exit $rc
