# round 5: pipelined host path, half-size end sub-batches A/B
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05k
mkdir -p $O
DS=/tmp/nym_1m.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > $O/gen.txt 2>&1 || exit $?
for r in 1 2; do for half in 1 0; do for sub in 262144 196608; do
  echo "== half $half sub $sub" >> $O/host_ab.txt
  PV_PIPE_TRACE=1 PV_PIPE_HALF_ENDS=$half PV_PIPE_SUB=$sub timeout -k 10 300 python -u tools/host_path_probe.py --dataset $DS --sizes 1048576 --reps 5 >> $O/host_ab.txt 2>&1 || exit $?
done; done; done
timeout -k 10 900 python -u -m pytest tests/test_gpu_host_path.py tests/test_gpu_abi.py -x -v --timeout 600 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
