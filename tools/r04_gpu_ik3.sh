#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04ik3
for r in 1 2; do
  timeout -k 10 200 python bench.py --legs ikfom --cpu-seconds 0 --pmc off --steps 20 > gpurun_out/r04ik3/pc1_$r.log 2>&1 || exit $?
  LIVO_LIB=fast-livo-noted_amd/lib/variants/ikpc0.so timeout -k 10 200 python bench.py --legs ikfom --cpu-seconds 0 --pmc off --steps 20 > gpurun_out/r04ik3/pc0_$r.log 2>&1 || exit $?
done
