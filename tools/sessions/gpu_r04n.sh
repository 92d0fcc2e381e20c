#!/bin/bash
# CPython fast-call binding of pv_verify_batch (plenum_amd/_fastcall.c) vs the ctypes path
# (PLENUM_AMD_NO_FASTCALL=1), same library: host-buffer latency A/B, then the whole GPU suite.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r04n
mkdir -p $O
for r in 1 2; do
  for v in fast ctypes; do
    if [ "$v" = ctypes ]; then export PLENUM_AMD_NO_FASTCALL=1; else unset PLENUM_AMD_NO_FASTCALL; fi
    timeout -k 10 120 python3 tools/lat_breakdown.py run 300 1,100,1000 > $O/$v.$r.json 2> $O/$v.$r.log || exit $?
    echo "$v $(cat $O/$v.$r.json)" >> $O/ab_fastcall.txt
  done
done
unset PLENUM_AMD_NO_FASTCALL
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_all.txt 2>&1 || exit $?
