# round 5: four-wave latency kernel, cached keys: [k](-A) on waves 2/3 beside the decompression
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05q
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_keycache.py tests/test_gpu_parity.py -x -v --timeout 600 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
DS=/tmp/nym_1m.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > $O/gen.txt 2>&1 || exit $?
for r in 1 2; do for lib in new pre; do
  if [ $lib = pre ]; then L=variants/pre_latcache/libplenum_verify.so; else L=indy-plenum_amd/plenum_amd/libplenum_verify.so; fi
  PLENUM_AMD_LIB=$L timeout -k 10 600 python3 bench.py --dataset $DS --no-cpu-baseline --no-config3 --no-ingress --no-multisig --no-straus --steps 10 --warmup 5 > $O/bench_$lib.$r.json 2> $O/bench_$lib.$r.log || exit $?
done; done
