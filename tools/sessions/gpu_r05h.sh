# round 5: full GPU suite; affine cached rows A/B (key cache); shared-table pipelined host path A/B
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05h
mkdir -p $O
DS=/tmp/nym_1m.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS > $O/gen.txt 2>&1 || exit $?
for r in 1 2; do
  for lib in new pre; do
    if [ $lib = pre ]; then L=variants/pre_affine/libplenum_verify.so; else L=indy-plenum_amd/plenum_amd/libplenum_verify.so; fi
    for m in fresh cached; do
      echo -n "$lib " >> $O/keycache_ab.txt
      PLENUM_AMD_LIB=$L timeout -k 10 300 python3 tools/keycache_probe.py --dataset $DS --mode $m --steps 20 >> $O/keycache_ab.txt 2>&1 || exit $?
    done
  done
done
for share in 1 0; do for sub in 65536 131072 262144; do
  echo "== share $share sub $sub" >> $O/host_ab.txt
  PV_PIPE_TRACE=1 PV_PIPE_SHARE=$share PV_PIPE_SUB=$sub timeout -k 10 300 python -u tools/host_path_probe.py --dataset $DS --sizes 1048576 --reps 5 >> $O/host_ab.txt 2>&1 || exit $?
done; done
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
