# round 5: fixed-base comb radix 2^26 (10 lookups, 38.7 GB) vs 2^24 (11 lookups, 10.7 GB): headline A/B
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05r
mkdir -p $O
DS=/tmp/nym_1m.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > $O/gen.txt 2>&1 || exit $?
for r in 1 2 3; do for lib in w26 base; do
  if [ $lib = w26 ]; then L=variants/w26/libplenum_verify.so; else L=indy-plenum_amd/plenum_amd/libplenum_verify.so; fi
  PLENUM_AMD_LIB=$L timeout -k 10 600 python3 bench.py --dataset $DS --no-cpu-baseline --no-config3 --no-ingress --no-multisig --no-straus --no-host-path --steps 20 --warmup 10 > $O/bench_$lib.$r.json 2> $O/bench_$lib.$r.log || exit $?
done; done
