#!/bin/bash
# round 6: the fused comb kernel's last-dispatched workgroups (last 1/4: variants/tail4, last 1/8:
# variants/tail8) at issue priority 1, against base: do the final round's young workgroups catch up?
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r06o
mkdir -p $O
AB_EXTRA="--no-config3 --sustain-s 0" timeout -k 10 1000 bash tools/ab_env.sh 4 "base:" "tail4:PLENUM_AMD_LIB=variants/tail4/libplenum_verify.so" "tail8:PLENUM_AMD_LIB=variants/tail8/libplenum_verify.so" > $O/ab_comb_ab_tail_prio.txt 2>&1 || exit $?
