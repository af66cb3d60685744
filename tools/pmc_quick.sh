#!/bin/bash
# Quick rocprofv3 --pmc passes over tools/knn_probe.py (the bench's batch, one
# step), k_iekf_eval dispatches only: instruction mix, waits, traffic.
# usage: tools/pmc_quick.sh <out_dir>    (summarise: python tools/pmc_summary.py <out_dir> tag out.json)
set -o pipefail
OUT=$1
cd /tmp && export TMPDIR=/tmp
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA" \
         "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex "k_iekf_eval" --output-format csv \
      -d $OUT/pass$i -o pmc -- python3 $GRAFT_REPO_ROOT/tools/knn_probe.py --steps 1 || exit $?
done
