#!/bin/bash
# round 6 mid-round: the whole GPU suite, smoke, the driver's bench command
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r06d
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.log || exit $?
