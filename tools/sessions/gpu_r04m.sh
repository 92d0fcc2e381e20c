#!/bin/bash
# [s2]B's 16 comb additions moved from wave 1 to waves 2 and 3 (four-wave latency kernel): latency
# parity, phase trace and host-buffer latency against the previous commit's build (variants/latprev).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r04m
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_robustness.py -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
for v in lattrace latprevtrace; do
  PLENUM_AMD_LIB=variants/$v/libplenum_verify.so timeout -k 10 120 python3 tools/lat_trace.py 50 > $O/trace_$v.txt 2>&1 || exit $?
done
rm -rf gpurun_out/ablat
SIZES=1,100,256 timeout -k 10 400 bash tools/ab_latency.sh base latprev > $O/ab_latency.txt 2>&1 || exit $?
cp -r gpurun_out/ablat $O/
