#!/bin/bash
# Separate rocprofv3 --pmc passes over a short bench run (counters only with
# --kernel-trace-free collection; never combined with sys/runtime traces).
# usage: tools/pmc_passes.sh <out_dir> [bench args...]
set -o pipefail
OUT=$1; shift
ARGS="$@"
cd /tmp && export TMPDIR=/tmp
i=0
for P in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
         "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
         "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-include-regex "k_knn_leaf|k_knn_grid|k_hshare|k_solve" --output-format csv \
      -d $OUT/pass$i -o pmc -- python $GRAFT_REPO_ROOT/bench.py $ARGS || exit $?
done
