# round 5: host path with the key cache (wide rows) -- why slower than without?
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05p
mkdir -p $O
DS=/tmp/nym_1m.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > $O/gen.txt 2>&1 || exit $?
for cfg in "PV_KC_WIDE_KEYS=1024" "PV_KC_WIDE_KEYS=0" "PV_KC_WIDE_KEYS=1024 PV_PIPE_SUB=524288"; do
  echo "== $cfg" >> $O/ab.txt
  env $cfg PV_PIPE_TRACE=1 timeout -k 10 300 python -u tools/host_path_probe.py --dataset $DS --sizes 1048576 --reps 5 --cache 2048 >> $O/ab.txt 2>&1 || exit $?
done
PV_PIPE_SUB=262144 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/trace -o run -- python3 tools/host_path_probe.py --dataset $DS --sizes 1048576 --reps 3 --cache 2048 > $O/probe_traced.txt 2> $O/trace.log || exit $?
python3 tools/copy_overlap.py $O/trace/run_results.db --calls 1 --events --all-kernels > $O/overlap.txt 2>&1 || exit $?
