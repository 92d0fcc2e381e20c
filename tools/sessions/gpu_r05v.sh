# round 5: the bench's host-path legs with the pipeline trace (arena slower inside bench.py than in the probe); then with the pinned block cache
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05v
mkdir -p $O
DS=/tmp/nym_1m.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > $O/gen.txt 2>&1 || exit $?
PV_PIPE_TRACE=1 timeout -k 10 600 python3 bench.py --dataset $DS --no-cpu-baseline --no-config3 --no-ingress --no-multisig --no-straus --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.log || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_host_path.py -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
