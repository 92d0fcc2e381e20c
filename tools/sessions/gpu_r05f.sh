# round 5: untraced pipeline timelines (PV_PIPE_TRACE) over copy-stream priority x lookahead x sub-batch size
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05f
mkdir -p $O
DS=/tmp/nym_1m.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > $O/gen.txt 2>&1 || exit $?
for prio in 1 0; do for la in 1 0; do for sub in 131072 262144; do
  echo "== prio $prio lookahead $la sub $sub" >> $O/ab.txt
  PV_PIPE_TRACE=1 PV_CSTREAM_PRIO=$prio PV_PIPE_LOOKAHEAD=$la PV_PIPE_SUB=$sub timeout -k 10 300 python -u tools/host_path_probe.py --dataset $DS --sizes 1048576 --reps 3 >> $O/ab.txt 2>&1 || exit $?
done; done; done
