#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04z
for s0 in 0 24; do
  LIVO_LIB=fast-livo-noted_amd/lib/variants/evprof.so timeout -k 10 200 python tools/eval_prof.py --seed0 $s0 > gpurun_out/r04z/evprof_seed$s0.txt 2>&1 || exit $?
done
