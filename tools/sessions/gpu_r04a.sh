set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r04a
timeout -k 10 900 python -u -m pytest tests/test_gpu_abi.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04a/gpu_tests_new.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-ingress --no-multisig --no-host-path > gpurun_out/r04a/bench.json 2> gpurun_out/r04a/bench.log
