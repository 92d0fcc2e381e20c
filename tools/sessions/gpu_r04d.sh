#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r04d
mkdir -p $O
timeout -k 10 900 bash tools/ab_env.sh 2 "base:" "pad41k:PV_PREP_LDS_PAD=41984" "pad54k:PV_PREP_LDS_PAD=54272" > $O/ab_pad.txt 2>&1 || exit $?
DS=/tmp/nym_ab.npz
PV_PREP_LDS_PAD=41984 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 bench.py --dataset $DS --no-cpu-baseline --no-host-path --no-ingress --no-multisig --no-straus --no-config3 --steps 20 --warmup 5 > $O/bench_traced.json 2> $O/trace.log || exit $?
