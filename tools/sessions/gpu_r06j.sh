#!/bin/bash
# round 6: encode at 8 points per lane with the dual-row wave inversion (two tree products, five column
# terms per lane): GPU suite, then interleaved A/B against the four-row inversion (variants/dual0)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r06j
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
AB_EXTRA="--no-config3 --sustain-s 0" timeout -k 10 900 bash tools/ab_env.sh 3 "base:" "dual0:PLENUM_AMD_LIB=variants/dual0/libplenum_verify.so" > $O/ab_enc_dual.txt 2>&1 || exit $?
timeout -k 10 700 bash tools/ab_straus.sh 2 base dual0 > $O/ab_straus_enc_dual.txt 2>&1 || exit $?
