#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04r
LIVO_LIB=fast-livo-noted_amd/lib/variants/ikprof.so timeout -k 10 200 python tools/ik_prof.py > gpurun_out/r04r/ik_prof.txt 2>&1 || exit $?
for rf in 0.5 2.0; do
  LIVO_DYN_REBASE=$rf timeout -k 10 300 python bench.py --legs ikd --cpu-seconds 0 --pmc off --steps 2 > gpurun_out/r04r/ikd_rebase_$rf.log 2>&1 || exit $?
done
