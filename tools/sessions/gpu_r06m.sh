#!/bin/bash
# round 6: pipelined host path, first/last piece size (PV_PIPE_END) 131072 (default) / 65536 / 32768 /
# 16384, interleaved, pageable and arena inputs at 1M requests; PV_PIPE_TRACE piece timings for each
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r06m
mkdir -p $O
DS=/tmp/nym_ab.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > /dev/null || exit $?
for r in 1 2 3; do
  for e in 131072 65536 32768 16384; do
    echo "== end $e round $r" >> $O/ab_pipe_end.txt
    PV_PIPE_END=$e timeout -k 10 200 python3 tools/host_path_probe.py --dataset $DS --sizes 1048576 --reps 7 >> $O/ab_pipe_end.txt 2>> $O/ab_pipe_end.log || exit $?
  done
done
echo "== traces" >> $O/ab_pipe_end.txt
for e in 131072 32768; do
  echo "== trace end $e" >> $O/ab_pipe_trace.txt
  PV_PIPE_TRACE=1 PV_PIPE_END=$e timeout -k 10 200 python3 tools/host_path_probe.py --dataset $DS --sizes 1048576 --reps 3 >> $O/ab_pipe_trace.txt 2>&1 || exit $?
done
