# round 5: lazy ev_launch_done recording on the engine's own stream (PV_LAZY_LAUNCH_EVENT) A/B + full GPU suite
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05ac
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
DS=/tmp/nym_1m.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > $O/gen.txt 2>&1 || exit $?
for r in 1 2 3; do for lz in 1 0; do
  PV_LAZY_LAUNCH_EVENT=$lz timeout -k 10 600 python3 bench.py --dataset $DS --no-cpu-baseline --no-config3 --no-ingress --no-multisig --no-straus --no-host-path --steps 20 --warmup 10 > $O/bench_lz$lz.$r.json 2> $O/bench_lz$lz.$r.log || exit $?
done; done
PV_LAZY_LAUNCH_EVENT=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace_lz1 -o run -- python3 bench.py --dataset $DS --no-cpu-baseline --no-config3 --no-ingress --no-multisig --no-straus --no-host-path --steps 10 --warmup 3 > $O/trace_lz1.log 2>&1 || exit $?
