#!/bin/bash
# round 4: request-order comb prep + direct fill -- comb-path parity, A/B (slot-order prep, fstream fill,
# prep occupancy cap), PMC FETCH/WRITE of the prep kernels
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_abi.py tests/test_gpu_parity.py tests/test_gpu_keycache.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
SL=variants/slotorder/libplenum_verify.so
ND=variants/nodirect/libplenum_verify.so
P=PV_PREP_LDS_PAD=41984
timeout -k 10 900 bash tools/ab_env.sh 2 "req_pad:$P" "slot_pad:$P PLENUM_AMD_LIB=$SL" "nodirect_pad:$P PLENUM_AMD_LIB=$ND" "req:" > $O/ab_req.txt 2>&1 || exit $?
DS=/tmp/nym_ab.npz
B="python3 bench.py --dataset $DS --no-cpu-baseline --no-host-path --no-ingress --no-multisig --no-straus --no-config3 --steps 3 --warmup 1"
for v in req slot; do
  if [ $v = slot ]; then export PLENUM_AMD_LIB=$SL; else unset PLENUM_AMD_LIB; fi
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_${v}_f -o run -- $B > /dev/null 2> $O/pmc_${v}_f.log || exit $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_${v}_w -o run -- $B > /dev/null 2> $O/pmc_${v}_w.log || exit $?
done
