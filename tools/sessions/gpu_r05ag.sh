# round 5: full GPU suite + smoke at the final code (encode group helpers)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05ag
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
