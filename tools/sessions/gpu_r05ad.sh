# round 5: msm lanes regrouped per tile by window count (PV_MSM_SORT) A/B + parity
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05ad
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_robustness.py -x -q --timeout 600 --timeout-method thread > $O/parity.txt 2>&1 || exit $?
DS=/tmp/nym_1m.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > $O/gen.txt 2>&1 || exit $?
for r in 1 2 3; do for lib in sort nosort; do
  if [ $lib = nosort ]; then L=variants/nosort/libplenum_verify.so; else L=indy-plenum_amd/plenum_amd/libplenum_verify.so; fi
  PLENUM_AMD_LIB=$L timeout -k 10 600 python3 bench.py --dataset $DS --no-cpu-baseline --no-ingress --no-multisig --no-host-path --steps 10 --warmup 5 > $O/bench_$lib.$r.json 2> $O/bench_$lib.$r.log || exit $?
done; done
