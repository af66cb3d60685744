#!/bin/bash
# Instruction-cache counters of the fused evaluation kernel over tools/knn_probe.py
# usage: tools/pmc_icache.sh <out_dir>
set -o pipefail
OUT=$1
cd /tmp && export TMPDIR=/tmp
i=0
for P in "SQC_ICACHE_HITS SQC_ICACHE_MISSES" "SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ" "SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $P --kernel-include-regex "k_iekf_eval" --output-format csv \
      -d $OUT/pass$i -o pmc -- python3 $GRAFT_REPO_ROOT/tools/knn_probe.py || exit $?
done
