# round 5: Straus table kernel at 3 waves/SIMD (168 VGPRs, 264 B spilled) vs 2 (256 VGPRs)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05ae
mkdir -p $O
DS=/tmp/nym_1m.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > $O/gen.txt 2>&1 || exit $?
PLENUM_AMD_LIB=variants/tb3/libplenum_verify.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/parity_tb3.txt 2>&1 || exit $?
for r in 1 2 3; do for lib in tb3 base; do
  if [ $lib = tb3 ]; then L=variants/tb3/libplenum_verify.so; else L=indy-plenum_amd/plenum_amd/libplenum_verify.so; fi
  PLENUM_AMD_LIB=$L timeout -k 10 600 python3 bench.py --dataset $DS --no-cpu-baseline --no-config3 --no-ingress --no-multisig --no-host-path --steps 10 --warmup 5 > $O/bench_$lib.$r.json 2> $O/bench_$lib.$r.log || exit $?
done; done
