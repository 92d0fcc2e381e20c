# round 5: host path arena vs pageable, without and with the key cache, alternating calls, pipeline trace
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05u
mkdir -p $O
DS=/tmp/nym_1m.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > $O/gen.txt 2>&1 || exit $?
PV_PIPE_TRACE=1 timeout -k 10 300 python3 -u tools/host_path_probe.py --dataset $DS --sizes 1048576 --reps 7 > $O/nocache.txt 2> $O/nocache_trace.txt || exit $?
PV_PIPE_TRACE=1 timeout -k 10 300 python3 -u tools/host_path_probe.py --dataset $DS --sizes 1048576 --reps 7 --cache 2048 > $O/cache.txt 2> $O/cache_trace.txt || exit $?
