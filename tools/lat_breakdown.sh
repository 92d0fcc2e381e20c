set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/latbd -o run -- python3 $R/tools/lat_breakdown.py run > $R/gpurun_out/latbd_run.json 2> $R/gpurun_out/latbd.log || exit $?
DB=$(ls $R/gpurun_out/latbd/*/run_results.db $R/gpurun_out/latbd/*.db 2>/dev/null | head -1)
python3 $R/tools/lat_breakdown.py analyze $DB > $R/gpurun_out/latbd.txt 2>&1; cat $R/gpurun_out/latbd_run.json $R/gpurun_out/latbd.txt
