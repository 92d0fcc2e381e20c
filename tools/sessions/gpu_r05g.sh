# round 5: shared comb tables across the pipelined sub-batches: parity + host-path A/B
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05g
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_host_path.py tests/test_gpu_keycache.py -x -v --timeout 600 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
DS=/tmp/nym_1m.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > $O/gen.txt 2>&1 || exit $?
for share in 1 0; do for sub in 65536 131072 262144; do
  echo "== share $share sub $sub" >> $O/ab.txt
  PV_PIPE_TRACE=1 PV_PIPE_SHARE=$share PV_PIPE_SUB=$sub timeout -k 10 300 python -u tools/host_path_probe.py --dataset $DS --sizes 1048576 --reps 5 >> $O/ab.txt 2>&1 || exit $?
done; done
