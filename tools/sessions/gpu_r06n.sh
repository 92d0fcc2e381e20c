#!/bin/bash
# round 6: the split comb form again at the round-6 pipeline (comb_b beside the fill, then comb_a:
# variants/fused0) and [S]B from the chunk start on its own stream (variants/bearly), against the fused
# kernel (base)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r06n
mkdir -p $O
AB_EXTRA="--sustain-s 0" timeout -k 10 1100 bash tools/ab_env.sh 3 "base:" "fused0:PLENUM_AMD_LIB=variants/fused0/libplenum_verify.so" "bearly:PLENUM_AMD_LIB=variants/bearly/libplenum_verify.so" > $O/ab_comb_form.txt 2>&1 || exit $?
