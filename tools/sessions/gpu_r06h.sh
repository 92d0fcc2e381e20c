#!/bin/bash
# round 6: encode kernel with the wave-wide limb-parallel inversion (PV_ENC_WAVE_INV=1): GPU parity
# suites (every verdict passes through the encode), verify_one, then interleaved A/B against the
# per-lane exponentiation chain (variants/encinv0) on the headline and the Straus path
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r06h
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
AB_EXTRA="--no-config3 --sustain-s 0" timeout -k 10 900 bash tools/ab_env.sh 3 "base:" "encinv0:PLENUM_AMD_LIB=variants/encinv0/libplenum_verify.so" > $O/ab_encinv.txt 2>&1 || exit $?
timeout -k 10 700 bash tools/ab_straus.sh 2 base encinv0 > $O/ab_straus_encinv.txt 2>&1 || exit $?
