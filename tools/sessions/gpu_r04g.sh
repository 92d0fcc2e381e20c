#!/bin/bash
# round 4: two chunk lanes with more hardware queues per process (HIP default 4)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r04g
mkdir -p $O
DS4=/tmp/nym_4m.npz
timeout -k 10 300 python3 tools/nym_workload.py --out $DS4 --n 4194304 > /dev/null || exit $?
for r in 1 2; do
  for v in "lanes_q8:GPU_MAX_HW_QUEUES=8" "one_q8:GPU_MAX_HW_QUEUES=8 PV_LANES=1" "lanes_q4:GPU_MAX_HW_QUEUES=4" "one_q4:GPU_MAX_HW_QUEUES=4 PV_LANES=1"; do
    name="${v%%:*}"; envs="${v#*:}"
    env $envs timeout -k 10 300 python3 bench.py --dataset $DS4 --per-gpu 4194304 --no-cpu-baseline --no-host-path --no-ingress --no-straus --no-config3 --no-multisig --steps 10 --warmup 3 > $O/b4m_$name.$r.json 2> $O/b4m_$name.$r.log || exit $?
    python3 -c "import json; d=json.loads(open('$O/b4m_$name.$r.json').read().strip().splitlines()[-1]); print('$name 4M', round(d['value']/1e6,1), 'M/s', d['ms_per_step'], 'ms', d['verdicts_ok'])"
  done
done > $O/ab_lanes_queues.txt
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run -- python3 bench.py --dataset $DS4 --per-gpu 4194304 --no-cpu-baseline --no-host-path --no-ingress --no-straus --no-config3 --no-multisig --steps 4 --warmup 2 > $O/traced.json 2> $O/trace.log || exit $?
