# round 5: kernel + memory-copy trace of the pipelined host path at several sub-batch sizes
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05c
mkdir -p $O
DS=/tmp/nym_1m.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > $O/gen.txt 2>&1 || exit $?
for sub in 262144 65536; do
  PV_PIPE_SUB=$sub timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/trace_$sub -o run -- python3 tools/host_path_probe.py --dataset $DS --sizes 1048576 --reps 3 > $O/probe_$sub.txt 2> $O/trace_$sub.log || exit $?
  python3 tools/copy_overlap.py $O/trace_$sub/run_results.db --calls 2 --events > $O/overlap_$sub.txt 2>&1 || exit $?
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_host_path.py tests/test_gpu_abi.py -x -v --timeout 600 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
