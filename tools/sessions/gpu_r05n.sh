# round 5: wide (radix-65536) cached key rows: A/B on the cached headline batch + GPU tests
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05n
mkdir -p $O
DS=/tmp/nym_1m.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > $O/gen.txt 2>&1 || exit $?
for r in 1 2; do
  for wide in 1024 0; do
    echo -n "wide=$wide " >> $O/keycache_ab.txt
    PV_KC_WIDE_KEYS=$wide timeout -k 10 300 python3 tools/keycache_probe.py --dataset $DS --mode cached --steps 20 >> $O/keycache_ab.txt 2>&1 || exit $?
  done
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_keycache.py tests/test_gpu_configs.py -x -v --timeout 600 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
