#!/bin/bash
# round 6: the driver's default bench command at the encode change (every leg incl. the unbatched drop-in
# through verify_one) and smoke()
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r06l
mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 900 python3 bench.py > $O/bench.json 2> $O/bench.log || exit $?
