set -o pipefail
export TMPDIR=/tmp
DS=/tmp/nym_1m.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > /dev/null || exit $?
for v in base norank; do
  if [ $v = base ]; then unset PLENUM_AMD_LIB; else export PLENUM_AMD_LIB=variants/$v/libplenum_verify.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ins_$v -o run -- python3 bench.py --dataset $DS --no-cpu-baseline --no-host-path --no-config3 --no-straus --no-ingress --no-multisig --steps 10 --warmup 2 > gpurun_out/ins_$v.json 2> gpurun_out/ins_$v.log || exit $?
  grep -h "insert\|assign\|scatter" gpurun_out/ins_$v/*/*stats.csv gpurun_out/ins_$v/*stats.csv 2>/dev/null | cut -c1-150
done
