# round 5: pipelined host path after the priority copy stream + lookahead enqueue
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05e
mkdir -p $O
DS=/tmp/nym_1m.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > $O/gen.txt 2>&1 || exit $?
for sub in 131072 65536 262144 131072; do
  PV_PIPE_SUB=$sub timeout -k 10 300 python -u tools/host_path_probe.py --dataset $DS --sizes 262144,1048576 --reps 7 > $O/host_probe_$sub.txt 2>&1 || exit $?
done
PV_PIPE_SUB=131072 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/trace_131072 -o run -- python3 tools/host_path_probe.py --dataset $DS --sizes 1048576 --reps 3 > $O/probe_traced.txt 2> $O/trace.log || exit $?
python3 tools/copy_overlap.py $O/trace_131072/run_results.db --calls 2 --events > $O/overlap_131072.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_host_path.py -x -v --timeout 600 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
