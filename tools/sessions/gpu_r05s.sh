# round 5: pipelined shared tables with one-off keys; drop-in per-call with auto cache
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05s
mkdir -p $O
true
DS=/tmp/nym_1m.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > $O/gen.txt 2>&1 || exit $?
timeout -k 10 600 python3 bench.py --no-config3 --no-multisig --no-straus --steps 10 --warmup 5 > $O/bench.json 2> $O/bench.log || exit $?
