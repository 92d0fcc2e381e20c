# round 5: kernel + copy trace of the shared-table pipelined host call (sub 65536) to see which kernels slow
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05j
mkdir -p $O
DS=/tmp/nym_1m.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > $O/gen.txt 2>&1 || exit $?
PV_PIPE_SUB=65536 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/trace -o run -- python3 tools/host_path_probe.py --dataset $DS --sizes 1048576 --reps 3 --no-arena > $O/probe.txt 2> $O/trace.log || exit $?
python3 tools/copy_overlap.py $O/trace/run_results.db --calls 1 --events --all-kernels > $O/overlap.txt 2>&1 || exit $?
