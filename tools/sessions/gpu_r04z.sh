#!/bin/bash
# Closed-form signed-digit recodings (sc_recode16 / 256 / 65536 as (a + M) xor M): parity, latency
# trace, host-buffer latency and the headline / configs[2] / Straus legs against the previous commit
# (variants/latprev9), interleaved on one box, then the whole GPU suite.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r04z
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_robustness.py -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
PLENUM_AMD_LIB=variants/lattrace/libplenum_verify.so timeout -k 10 120 python3 tools/lat_trace.py 50 > $O/trace_lattrace.txt 2>&1 || exit $?
rm -rf gpurun_out/ablat
SIZES=1,100,1000 timeout -k 10 400 bash tools/ab_latency.sh base latprev9 > $O/ab_latency.txt 2>&1 || exit $?
cp -r gpurun_out/ablat $O/
DS=/tmp/nym_ab.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > /dev/null || exit $?
for r in 1 2; do
  for v in base latprev9; do
    if [ "$v" = base ]; then unset PLENUM_AMD_LIB; else export PLENUM_AMD_LIB=variants/$v/libplenum_verify.so; fi
    timeout -k 10 300 python3 bench.py --dataset $DS --steps 20 --warmup 5 --no-cpu-baseline --no-host-path --no-ingress \
      --no-multisig --no-single-process > $O/head_$v.$r.json 2> $O/head_$v.$r.log || exit $?
    python3 -c "import json; d=json.load(open('$O/head_$v.$r.json')); c=d.get('config3',{}); s=d.get('straus_path',{}); print('$v', d['value'], d['ms_per_step'], c.get('value'), s.get('value'))" >> $O/ab_headline.txt || exit $?
  done
done
unset PLENUM_AMD_LIB
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_all.txt 2>&1 || exit $?
