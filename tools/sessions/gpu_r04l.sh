#!/bin/bash
# Final latency form (vector SHA, 53-bit split, y-only chains, dual-row decompression): latency parity,
# phase trace, host-buffer latency and the headline, each A/B against the session-start build
# (variants/lathead), interleaved on one box.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r04l
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_robustness.py -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
for v in lattrace latheadtrace; do
  PLENUM_AMD_LIB=variants/$v/libplenum_verify.so timeout -k 10 120 python3 tools/lat_trace.py 50 > $O/trace_$v.txt 2>&1 || exit $?
done
rm -rf gpurun_out/ablat
SIZES=1,100,1000 timeout -k 10 400 bash tools/ab_latency.sh base lathead > $O/ab_latency.txt 2>&1 || exit $?
cp -r gpurun_out/ablat $O/
DS=/tmp/nym_ab.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > /dev/null || exit $?
for r in 1 2; do
  for v in base lathead; do
    if [ "$v" = base ]; then unset PLENUM_AMD_LIB; else export PLENUM_AMD_LIB=variants/$v/libplenum_verify.so; fi
    timeout -k 10 300 python3 bench.py --dataset $DS --steps 20 --warmup 5 --no-cpu-baseline --no-host-path --no-ingress \
      --no-multisig --no-straus --no-single-process > $O/head_$v.$r.json 2> $O/head_$v.$r.log || exit $?
    python3 -c "import json,sys; d=json.load(open('$O/head_$v.$r.json')); c=d.get('config3',{}); print('$v', d['value'], d['ms_per_step'], c.get('value'), c.get('ms_per_step'))" >> $O/ab_headline.txt || exit $?
  done
done
