#!/bin/bash
# round 6: encode batch per lane with the wave inversion: 16 (base) vs 8 (variants/enc8) vs 4 (variants/enc4)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r06i
mkdir -p $O
AB_EXTRA="--no-config3 --sustain-s 0" timeout -k 10 900 bash tools/ab_env.sh 3 "base:" "enc8:PLENUM_AMD_LIB=variants/enc8/libplenum_verify.so" "enc4:PLENUM_AMD_LIB=variants/enc4/libplenum_verify.so" > $O/ab_enc_batch.txt 2>&1 || exit $?
timeout -k 10 700 bash tools/ab_straus.sh 2 base enc8 enc4 > $O/ab_straus_enc_batch.txt 2>&1 || exit $?
