#!/bin/bash
# round 4: front-window A/B (fill occupancy, chain parts) on the fused comb build
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 900 bash tools/ab_config3.sh base fill3 fill4 parts2 parts4 > $O/ab_front.txt 2>&1 || exit $?
