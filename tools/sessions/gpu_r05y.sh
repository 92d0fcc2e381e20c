# round 5: host-path GPU tests with the pinned block cache
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05y
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_host_path.py tests/test_gpu_abi.py -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
