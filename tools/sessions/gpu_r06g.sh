#!/bin/bash
# round 6: A/B of the comb_ab [S]B phase at issue priority 2 (younger waves first: equalised progress,
# shorter launch tail?) with the launch shape from the stamps of both
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r06g
mkdir -p $O
DS=/tmp/nym_ab.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > /dev/null || exit $?
for l in clock prio2clock; do
  PLENUM_AMD_LIB=variants/$l/libplenum_verify.so timeout -k 10 120 python3 tools/clock_probe.py --dataset $DS --label $l >> $O/shape.jsonl 2>> $O/shape.log || exit $?
done
AB_EXTRA="--no-config3 --sustain-s 0" timeout -k 10 900 bash tools/ab_env.sh 3 "base:" "prio2:PLENUM_AMD_LIB=variants/prio2/libplenum_verify.so" > $O/ab_prio.txt 2>&1 || exit $?
