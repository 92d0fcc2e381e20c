# round 5: full bench line + host-path trace evidence (kernels + copies) at the current code
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05l
mkdir -p $O
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.log || exit $?
DS=/tmp/nym_1m.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > $O/gen.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/trace -o run -- python3 tools/host_path_probe.py --dataset $DS --sizes 1048576 --reps 5 > $O/probe_traced.txt 2> $O/trace.log || exit $?
python3 tools/copy_overlap.py $O/trace/run_results.db --calls 3 --events > $O/overlap.txt 2>&1 || exit $?
