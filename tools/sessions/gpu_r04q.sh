#!/bin/bash
# Four-wave kernel: the waves' parts converted to cached form before barrier 2 (off wave 0's final
# chain); leaner Python wrapper. Latency parity, trace and host-buffer latency against the previous
# commit's library (variants/latprev3), then the whole GPU suite.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r04q
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_robustness.py -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
for v in lattrace latprev3trace; do
  PLENUM_AMD_LIB=variants/$v/libplenum_verify.so timeout -k 10 120 python3 tools/lat_trace.py 50 > $O/trace_$v.txt 2>&1 || exit $?
done
rm -rf gpurun_out/ablat
SIZES=1,100,1000 timeout -k 10 400 bash tools/ab_latency.sh base latprev3 > $O/ab_latency.txt 2>&1 || exit $?
cp -r gpurun_out/ablat $O/
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_all.txt 2>&1 || exit $?
