#!/bin/bash
# round 6 end evidence: full GPU suite, smoke, the driver's bench command, kernel trace + PMC passes
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
TAG=${TAG:-r06end}
O=gpurun_out/$TAG
mkdir -p $O
echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null) nproc: $(nproc)" > $O/host_cpus.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.log || exit $?
timeout -k 10 900 bash tools/profile_round.sh $TAG > $O/profile.log 2>&1 || exit $?
