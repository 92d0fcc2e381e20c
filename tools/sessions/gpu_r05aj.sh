# round 5: the encode's inversion with plain-C++ squarings (PV_ENC_ILP=1, variants/encilp) vs column asm
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05aj
mkdir -p $O
PLENUM_AMD_LIB=variants/encilp/libplenum_verify.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 600 --timeout-method thread > $O/parity_encilp.txt 2>&1 || exit $?
DS=/tmp/nym_1m.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > $O/gen.txt 2>&1 || exit $?
for r in 1 2 3; do for lib in encilp main; do
  if [ $lib = main ]; then L=indy-plenum_amd/plenum_amd/libplenum_verify.so; else L=variants/$lib/libplenum_verify.so; fi
  PLENUM_AMD_LIB=$L timeout -k 10 600 python3 bench.py --dataset $DS --no-cpu-baseline --no-ingress --no-multisig --no-config3 --no-host-path --steps 20 --warmup 10 > $O/bench_$lib.$r.json 2> $O/bench_$lib.$r.log || exit $?
done; done
