#!/bin/bash
# round 6: the step-time ramp from an idle GPU (clock stamps per step); A/B of the fill's wave priority
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r06c
mkdir -p $O
DS=/tmp/nym_ab.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > /dev/null || exit $?
for r in 1 2; do
  PLENUM_AMD_LIB=variants/clock/libplenum_verify.so timeout -k 10 120 python3 tools/clock_probe.py --dataset $DS --ramp --label ramp$r >> $O/ramp.jsonl 2>> $O/ramp.log || exit $?
done
AB_EXTRA="--no-config3" timeout -k 10 900 bash tools/ab_env.sh 3 "base:" "fillprio1:PLENUM_AMD_LIB=variants/fillprio1/libplenum_verify.so" "fillprio3:PLENUM_AMD_LIB=variants/fillprio3/libplenum_verify.so" > $O/ab_fillprio.txt 2>&1 || exit $?
exit 0
