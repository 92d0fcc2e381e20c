# round 5: encode with 16 points per lane, two groups of 8 under one inversion (PV_ENC_BATCH_N=16) vs 8
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05af
mkdir -p $O
PLENUM_AMD_LIB=variants/enc16b/libplenum_verify.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 600 --timeout-method thread > $O/parity_enc16b.txt 2>&1 || exit $?
DS=/tmp/nym_1m.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > $O/gen.txt 2>&1 || exit $?
for r in 1 2 3; do for lib in enc16b base; do
  if [ $lib = enc16b ]; then L=variants/enc16b/libplenum_verify.so; else L=indy-plenum_amd/plenum_amd/libplenum_verify.so; fi
  PLENUM_AMD_LIB=$L timeout -k 10 600 python3 bench.py --dataset $DS --no-cpu-baseline --no-ingress --no-multisig --no-host-path --steps 20 --warmup 10 > $O/bench_$lib.$r.json 2> $O/bench_$lib.$r.log || exit $?
done; done
