# round 5: what slows the arena DMA in bench.py's cached host-path leg (tools/host_path_bisect.py)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05w
mkdir -p $O
DS=/tmp/nym_1m.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > $O/gen.txt 2>&1 || exit $?
i=0
for ops in "host cache host dev host" "host lat host cache host" "host auto nocache cache host" "host cache lat host dev host"; do
  i=$((i+1))
  echo "== $ops" > $O/b$i.txt
  PV_PIPE_TRACE=1 timeout -k 10 300 python3 -u tools/host_path_bisect.py --dataset $DS $ops >> $O/b$i.txt 2> $O/b$i.trace || exit $?
done
