# round 5: Straus path with [k2 S]B forked onto the side stream beside the table kernel (PV_STRAUS_FORK_B) A/B + parity
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05aa
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 600 --timeout-method thread > $O/parity.txt 2>&1 || exit $?
DS=/tmp/nym_1m.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > $O/gen.txt 2>&1 || exit $?
for r in 1 2 3; do for fb in 1 0; do
  PV_STRAUS_FORK_B=$fb timeout -k 10 600 python3 bench.py --dataset $DS --no-cpu-baseline --no-config3 --no-ingress --no-multisig --no-host-path --steps 10 --warmup 5 > $O/bench_fb$fb.$r.json 2> $O/bench_fb$fb.$r.log || exit $?
done; done
