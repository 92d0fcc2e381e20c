# round 5: configs[2] with cached signers (affine rows) + the config tests + host path tests
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05m
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_host_path.py -x -v --timeout 600 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
