#!/bin/bash
# round 6: shape of the comb_ab launch from its per-workgroup stamps (diagnostic build)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r06f
mkdir -p $O
DS=/tmp/nym_ab.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > /dev/null || exit $?
PLENUM_AMD_LIB=variants/clock/libplenum_verify.so timeout -k 10 120 python3 tools/clock_probe.py --dataset $DS --label shape --dump $O/stamps.npz > $O/shape.jsonl 2> $O/shape.log || exit $?
