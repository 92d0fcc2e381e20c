#!/bin/bash
# Zero-copy calls no longer record the hand-over event (recorded lazily when another stream needs
# it): host-buffer latency A/B against the previous commit (variants/latprev2), then the GPU ABI /
# ordering tests and the whole GPU suite.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r04o
mkdir -p $O
rm -rf gpurun_out/ablat
SIZES=1,100,1000 timeout -k 10 400 bash tools/ab_latency.sh base latprev2 > $O/ab_latency.txt 2>&1 || exit $?
cp -r gpurun_out/ablat $O/
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_all.txt 2>&1 || exit $?
