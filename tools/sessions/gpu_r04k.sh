#!/bin/bash
# Latency path: 53-bit Lehmer split + y-only [2^68] chains in the four-wave kernel. Latency parity,
# phase traces (new vs HEAD build), host-buffer latency A/B against HEAD (variants/lathead).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r04k
mkdir -p $O
for v in s0 s1; do timeout -k 10 60 ./microbench/lp_split_lat_$v >> $O/lp_split_spec.txt || exit $?; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_robustness.py -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
for v in lattrace lattrace_vsha latheadtrace; do
  PLENUM_AMD_LIB=variants/$v/libplenum_verify.so timeout -k 10 120 python3 tools/lat_trace.py 50 > $O/trace_$v.txt 2>&1 || exit $?
done
rm -rf gpurun_out/ablat
SIZES=1,100,1000 timeout -k 10 400 bash tools/ab_latency.sh base lathead > $O/ab_latency.txt 2>&1 || exit $?
cp -r gpurun_out/ablat $O/
timeout -k 10 600 bash tools/ab_straus.sh 2 sc31 sc53 > $O/ab_straus.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_all.txt 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.log || exit $?
