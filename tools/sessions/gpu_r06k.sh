#!/bin/bash
# round 6: fused comb kernel in one-wave (variants/ab64) and two-wave (variants/ab128) workgroups against
# four-wave ones (base): a slot released per wave instead of per four
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r06k
mkdir -p $O
AB_EXTRA="--no-config3 --sustain-s 0" timeout -k 10 900 bash tools/ab_env.sh 3 "base:" "ab64:PLENUM_AMD_LIB=variants/ab64/libplenum_verify.so" "ab128:PLENUM_AMD_LIB=variants/ab128/libplenum_verify.so" > $O/ab_comb_ab_block.txt 2>&1 || exit $?
