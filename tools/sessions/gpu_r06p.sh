#!/bin/bash
# round 6: the encode's inversion chain shared by the workgroup's 4 waves (PV_ENC_WG_INV=1,
# variants/wginv): parity suite on that library, then interleaved A/B on the headline and Straus path
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r06p
mkdir -p $O
PLENUM_AMD_LIB=variants/wginv/libplenum_verify.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_wginv.txt 2>&1 || exit $?
AB_EXTRA="--no-config3 --sustain-s 0" timeout -k 10 900 bash tools/ab_env.sh 4 "base:" "wginv:PLENUM_AMD_LIB=variants/wginv/libplenum_verify.so" > $O/ab_encode_wg_inv.txt 2>&1 || exit $?
timeout -k 10 700 bash tools/ab_straus.sh 2 base wginv > $O/ab_encode_wg_inv_straus.txt 2>&1 || exit $?
