#!/bin/bash
# round 6: key-cache admission hardening on the GPU (keycache suite, ABI, host path with the test hook)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_keycache.py tests/test_abi.py tests/test_gpu_host_path.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
