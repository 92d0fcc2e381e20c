set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 120 ./microbench/h2d_bw > $O/h2d_bw.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/host_path_probe.py --sizes 262144,1048576 --reps 5 > $O/host_probe.txt 2>&1 || exit $?
