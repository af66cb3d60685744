#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04w
tools/ab_pool.sh 1 base@LIVO_BR_R=6 base@LIVO_BR_R=8 base@LIVO_BR_R=10 base@LIVO_BR_R=13 base@LIVO_BR_R=8,LIVO_BR_HA=1.5 base@LIVO_BR_R=8,LIVO_BR_HA=3 || exit $?
for r in 8 10; do
  LIVO_BR_R=$r timeout -k 10 300 python bench.py --legs config5 --steps 8 --cpu-seconds 0 --pmc off > gpurun_out/r04w/c5_r$r.log 2>&1 || exit $?
done
