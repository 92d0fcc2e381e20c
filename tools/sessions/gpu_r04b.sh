#!/bin/bash
# round 4: fused comb kernel -- full GPU suite, A/B against the two-kernel build, kernel trace
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
timeout -k 10 600 bash tools/ab_config3.sh base nofused > $O/ab_fused.txt 2>&1 || exit $?
DS=/tmp/nym_ab.npz
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 bench.py --dataset $DS --no-cpu-baseline --no-host-path --no-ingress --no-multisig --no-straus --no-config3 --steps 20 --warmup 5 > $O/bench_traced.json 2> $O/trace.log || exit $?
