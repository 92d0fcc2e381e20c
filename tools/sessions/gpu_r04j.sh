#!/bin/bash
# Scalar-unit SHA-512 in the latency kernels: latency parity, phase trace (scalar vs per-lane hash),
# host-buffer latency A/B against the per-lane build (variants/vsha).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r04j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_robustness.py -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
for v in lattrace lattrace0; do
  PLENUM_AMD_LIB=variants/$v/libplenum_verify.so timeout -k 10 120 python3 tools/lat_trace.py 50 > $O/trace_$v.txt 2>&1 || exit $?
done
SIZES=1,100,1000 timeout -k 10 400 bash tools/ab_latency.sh base vsha > $O/ab_latency.txt 2>&1 || exit $?
cp -r gpurun_out/ablat $O/
