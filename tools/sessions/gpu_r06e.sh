#!/bin/bash
# round 6: parity of the Straus loop that starts from the top window's A entry; A/B against the
# identity start (variants/topid) and the table built by additions only (variants/tabadd); the admission-hardening suites after the find/bump change
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r06e
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_robustness.py tests/test_gpu_keycache.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
timeout -k 10 1000 bash tools/ab_straus.sh 3 base topid tabadd > $O/ab_straus_topload_tabdbl.txt 2>&1 || exit $?
