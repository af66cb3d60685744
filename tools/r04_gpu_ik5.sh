#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04ik5
for r in 1 2; do
for v in base LIVO_IK_SIDE=0 LIVO_STREAM_GROUPS=4,LIVO_IK_SIDE=0 LIVO_STREAM_GROUPS=3 LIVO_STREAM_GROUPS=1; do
  e=""; [ "$v" != base ] && e=$(echo $v | tr ',' ' ')
  env $e timeout -k 10 200 python bench.py --legs ikfom --cpu-seconds 0 --pmc off --steps 20 > gpurun_out/r04ik5/${v}_$r.log 2>&1 || exit $?
done
done
