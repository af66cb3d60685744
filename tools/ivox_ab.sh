#!/bin/bash
# A/B of the two iVox search kernels on config-2 shapes (batch 8 and 1) and the per-frame pipeline.
set -e
for K in wave thread; do
  for B in 8 1; do
    echo "== LIVO_IVOX_KIND=$K batch $B"
    LIVO_IVOX_KIND=$K timeout -k 10 120 python tools/ivox_lab.py 1000000 100000 $B | grep -E "knn_first|batch"
  done
done
echo "== pipeline (auto)"
timeout -k 10 120 python tools/pipeline_lab.py | tail -1
