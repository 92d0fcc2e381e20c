#!/bin/bash
# round 4: two chunk lanes -- multi-chunk parity (configs[3], config5 shard, two chunks), A/B on a
# 4M-request (4-chunk) batch and the multisig leg, lanes vs one lane, and the 1M headline unchanged
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_abi.py -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
DS4=/tmp/nym_4m.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS4 --n 4194304 > /dev/null || exit $?
for r in 1 2; do
  for v in lanes one; do
    if [ $v = one ]; then export PV_LANES=1; else unset PV_LANES; fi
    timeout -k 10 300 python3 bench.py --dataset $DS4 --per-gpu 4194304 --no-cpu-baseline --no-host-path --no-ingress --no-straus --no-config3 --no-multisig --steps 10 --warmup 3 > $O/b4m_$v.$r.json 2> $O/b4m_$v.$r.log || exit $?
    python3 -c "import json; d=json.loads(open('$O/b4m_$v.$r.json').read().strip().splitlines()[-1]); print('$v 4M', round(d['value']/1e6,1), 'M/s', d['ms_per_step'], 'ms', d['verdicts_ok'])"
  done
done > $O/ab_lanes.txt
timeout -k 10 900 bash tools/ab_env.sh 1 "lanes:" "one:PV_LANES=1" >> $O/ab_lanes.txt 2>&1 || exit $?
