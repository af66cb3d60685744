#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04q
for k in 1.5 2 3 4; do
  LIVO_DYN_RUNS=0 LIVO_DYN_CELL_K=$k timeout -k 10 300 python bench.py --legs ikd --cpu-seconds 0 --pmc off --steps 2 > gpurun_out/r04q/ikd_k_$k.log 2>&1 || exit $?
done
