#!/bin/bash
# rocprofv3 --pmc passes over tools/knn_probe.py (the bench's batch), fused
# evaluation kernel only; one pass per counter set (MI355X_MICROARCH.md
# §rocprofv3 PMC slots: <= 8 SQ counters a pass).  Summarise with
#   python tools/pmc_summary.py <out_dir>
# usage: tools/pmc_eval.sh <out_dir>
set -o pipefail
OUT=$1
cd /tmp && export TMPDIR=/tmp
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR" \
         "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex "k_iekf_eval" --output-format csv \
      -d $OUT/pass$i -o pmc -- python3 $GRAFT_REPO_ROOT/tools/knn_probe.py || exit $?
done
