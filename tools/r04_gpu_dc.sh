#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04dc
timeout -k 10 600 python -u -m pytest tests/test_gpu_ikd_incr.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04dc/pytest_ikd_incr.log 2>&1 || exit $?
for f in 0 1.2 1.6 2.4; do
  LIVO_DYN_BOX_CELL=$f timeout -k 10 300 python bench.py --legs ikd --cpu-seconds 0 --pmc off --steps 2 > gpurun_out/r04dc/ikd_$f.log 2>&1 || exit $?
done
