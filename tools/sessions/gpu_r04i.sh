#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r04i
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_abi.py tests/test_gpu_keycache.py -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-ingress > $O/bench.json 2> $O/bench.log || exit $?
