#!/bin/bash
# Build an A/B variant of libplenum_verify.so with extra defines into variants/<name>/ (selected at
# run time with PLENUM_AMD_LIB=variants/<name>/libplenum_verify.so). Usage: build_variant.sh NAME -DX=1 ...
set -e
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/variants/$name
mkdir -p "$out/build"
cd "$root/indy-plenum_amd"
for f in pv_engine.hip pv_latency.hip pv_ingress.hip host_prep.cpp signing_json.cpp; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -Wall "$@" -c -o "$out/build/$f.o" "csrc/$f" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fPIC -shared -o "$out/libplenum_verify.so" "$out"/build/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf "$out/build"
echo "$out/libplenum_verify.so"
