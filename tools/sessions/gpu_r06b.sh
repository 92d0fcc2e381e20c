#!/bin/bash
# round 6: parity of the kstream fork after the scan; A/B fork-after-scan vs after-scatter; the
# in-kernel clock of comb_ab (diagnostic build) with the radix-2^16 [S]B lever; a kernel timeline
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r06b
mkdir -p $O
DS=/tmp/nym_ab.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > /dev/null || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_host_path.py tests/test_gpu_keycache.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_abi.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
AB_EXTRA="--no-config3" timeout -k 10 900 bash tools/ab_env.sh 3 "scan:" "scatter:PLENUM_AMD_LIB=variants/fork0/libplenum_verify.so" > $O/ab_fork.txt 2>&1 || exit $?
for r in 1 2 3; do
  PLENUM_AMD_LIB=variants/clock/libplenum_verify.so timeout -k 10 120 python3 tools/clock_probe.py --dataset $DS --label w24 >> $O/clock.jsonl 2>> $O/clock.log || exit $?
  PV_FORCE_BCOMB16=1 PLENUM_AMD_LIB=variants/clock/libplenum_verify.so timeout -k 10 120 python3 tools/clock_probe.py --dataset $DS --label w16 >> $O/clock.jsonl 2>> $O/clock.log || exit $?
  timeout -k 10 120 python3 tools/clock_probe.py --dataset $DS --label product >> $O/clock.jsonl 2>> $O/clock.log || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run -- python3 bench.py --dataset $DS --no-cpu-baseline --no-host-path --no-config3 --no-ingress --no-multisig --no-straus --steps 10 --warmup 5 > $O/bench_traced.json 2> $O/trace.log || exit $?
DB=$(find $O/trace -name "*.db" | head -1)
python3 tools/timeline.py $DB --steps 3 > $O/timeline.txt 2>&1
python3 tools/timeline.py $DB --summary > $O/timeline_summary.txt 2>&1
rm -f $DB
exit 0
