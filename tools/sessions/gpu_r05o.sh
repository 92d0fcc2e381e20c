# round 5: sampled automatic admission for large host batches + keycache suite + host path with cache
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05o
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_keycache.py -x -v --timeout 600 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
