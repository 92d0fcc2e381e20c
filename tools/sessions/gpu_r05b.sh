# round 5: host-fed path (arena + pipelined sub-batches): new GPU tests, sub-batch size A/B
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05b
mkdir -p $O
DS=/tmp/nym_1m.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > $O/gen.txt 2>&1 || exit $?
for sub in 131072 65536 262144; do
  PV_PIPE_SUB=$sub timeout -k 10 300 python -u tools/host_path_probe.py --dataset $DS --sizes 262144,1048576 --reps 7 > $O/host_probe_$sub.txt 2>&1 || exit $?
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_host_path.py tests/test_gpu_abi.py -x -v --timeout 600 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
