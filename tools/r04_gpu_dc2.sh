#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04dc2
timeout -k 10 600 python -u -m pytest tests/test_gpu_ikd_incr.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04dc2/pytest_ikd_incr.log 2>&1 || exit $?
for f in 2.6 0 2.0 3.4; do
  LIVO_DYN_BOX_CELL_MAX=$f timeout -k 10 300 python bench.py --legs ikd --cpu-seconds 0 --pmc off --steps 2 > gpurun_out/r04dc2/ikd_$f.log 2>&1 || exit $?
done
