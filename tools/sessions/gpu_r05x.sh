# round 5: NUMA placement of the pinned arena vs the GPU's node, in several fresh processes
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05x
mkdir -p $O
DS=/tmp/nym_1m.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > $O/gen.txt 2>&1 || exit $?
for i in 1 2 3 4 5 6; do
  timeout -k 10 120 python3 -u tools/numa_probe.py --dataset $DS >> $O/numa.txt 2>> $O/numa.err || exit $?
done
(lscpu; cat /sys/devices/system/node/node*/meminfo | grep -E "MemTotal|MemFree"; cat /proc/self/status | grep -i allowed) > $O/topo.txt 2>&1 || true
