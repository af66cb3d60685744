#!/bin/bash
# rocprofv3 --pmc passes over the probe batch given by the arguments (tools/knn_probe.py, e.g. --fresh or --config5;
# 10M-point map, 8 VoxelGrid scans of ~196k points, 4 stream groups), the
# k_iekf_eval dispatches only, one counter set per pass (MI355X_MICROARCH.md:
# FETCH_SIZE takes 3 TCC counters, WRITE_SIZE 2).
# usage: tools/pmc_c5.sh <abs out_dir> [probe args...]
#   (summarise: python tools/pmc_summary.py <out_dir> config5 out.json 4)
set -o pipefail
OUT=$1; shift
cd /tmp && export TMPDIR=/tmp
i=0
for P in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex "k_iekf_eval" --output-format csv \
      -d $OUT/pass$i -o pmc -- python3 $GRAFT_REPO_ROOT/tools/knn_probe.py --steps 4 "$@" || exit $?
done
