#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04iv2
for v in base LIVO_IVOX_KIND=wave LIVO_STREAM_GROUPS=4 LIVO_STREAM_GROUPS=1; do
  e=""; [ "$v" != base ] && e=$v
  env $e timeout -k 10 300 python bench.py --legs ivox --steps 10 --cpu-seconds 0 --pmc off > gpurun_out/r04iv2/$v.log 2>&1 || exit $?
done
