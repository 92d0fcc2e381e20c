# round 5: encode kernel templated on the batch (16 per lane for chunks >= 1M, 8 below; loads one point
# ahead) vs the previous 8-per-lane code (variants/enc8old); full GPU suite at this code
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05ai
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
DS=/tmp/nym_1m.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > $O/gen.txt 2>&1 || exit $?
for r in 1 2 3; do for lib in main enc8old; do
  if [ $lib = main ]; then L=indy-plenum_amd/plenum_amd/libplenum_verify.so; else L=variants/$lib/libplenum_verify.so; fi
  PLENUM_AMD_LIB=$L timeout -k 10 600 python3 bench.py --dataset $DS --no-cpu-baseline --no-ingress --no-multisig --no-config3 --steps 20 --warmup 10 > $O/bench_$lib.$r.json 2> $O/bench_$lib.$r.log || exit $?
done; done
