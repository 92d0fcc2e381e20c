# round 5: pipelined host path trace + new GPU tests + key-cache A/B (fresh vs cached tables) with PMC
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05d
mkdir -p $O
DS=/tmp/nym_1m.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > $O/gen.txt 2>&1 || exit $?
for sub in 262144 65536; do
  PV_PIPE_SUB=$sub timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/trace_$sub -o run -- python3 tools/host_path_probe.py --dataset $DS --sizes 1048576 --reps 3 > $O/probe_$sub.txt 2> $O/trace_$sub.log || exit $?
  python3 tools/copy_overlap.py $O/trace_$sub/run_results.db --calls 2 --events > $O/overlap_$sub.txt 2>&1 || exit $?
done
for m in fresh cached fresh cached; do
  timeout -k 10 300 python3 tools/keycache_probe.py --dataset $DS --mode $m >> $O/keycache_ab.txt 2>&1 || exit $?
done
for m in fresh cached; do
  i=0
  for ctr in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $ctr -d $O/pmc_${m}_$i -o run -- python3 tools/keycache_probe.py --dataset $DS --mode $m --steps 3 --warmup 1 > $O/pmc_${m}_$i.txt 2>&1 || exit $?
  done
  python3 tools/pmc_summary.py $O/pmc_$m.json $O/pmc_${m}_1 $O/pmc_${m}_2 $O/pmc_${m}_3 > /dev/null 2>&1 || true
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_host_path.py tests/test_gpu_abi.py -x -v --timeout 600 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
