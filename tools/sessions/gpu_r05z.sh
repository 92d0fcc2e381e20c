# round 5: device-scope release on the engine's stream-to-stream events (PV_EVENT_DEVSCOPE) A/B + parity; host-path tests
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05z
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_host_path.py tests/test_gpu_abi.py -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
PV_EVENT_DEVSCOPE=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 600 --timeout-method thread > $O/parity_devscope.txt 2>&1 || exit $?
DS=/tmp/nym_1m.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > $O/gen.txt 2>&1 || exit $?
for r in 1 2 3; do for ds in 1 0; do
  PV_EVENT_DEVSCOPE=$ds timeout -k 10 600 python3 bench.py --dataset $DS --no-cpu-baseline --no-config3 --no-ingress --no-multisig --no-straus --no-host-path --steps 20 --warmup 10 > $O/bench_ds$ds.$r.json 2> $O/bench_ds$ds.$r.log || exit $?
done; done
for ds in 1 0; do
  PV_EVENT_DEVSCOPE=$ds timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace_ds$ds -o run -- python3 bench.py --dataset $DS --no-cpu-baseline --no-config3 --no-ingress --no-multisig --no-straus --no-host-path --steps 10 --warmup 3 > $O/trace_ds$ds.log 2>&1 || exit $?
done
