#!/bin/bash
# Batch four-wave kernels with the SHA-512 inlined (126-138 VGPRs: four workgroups per CU), the
# one-request kernel keeping the call: parity, one-request trace, and the four-wave cutoff at
# 512 / 1,024 / 2,048 requests.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r04ad
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_robustness.py -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
PLENUM_AMD_LIB=variants/lattrace/libplenum_verify.so timeout -k 10 120 python3 tools/lat_trace.py 50 > $O/trace_lattrace.txt 2>&1 || exit $?
rm -rf gpurun_out/ablat
SIZES=1,100,384,512,768,1000,1536,2048 timeout -k 10 600 bash tools/ab_latency.sh base c1024 c2048 > $O/ab_cutoff.txt 2>&1 || exit $?
cp -r gpurun_out/ablat $O/
