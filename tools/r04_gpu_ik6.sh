#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04ik6
timeout -k 10 400 python -u -m pytest tests/test_gpu_ikfom.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04ik6/pytest_ikfom.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 200 python bench.py --legs ikfom --cpu-seconds 0 --pmc off --steps 20 > gpurun_out/r04ik6/bench_$r.log 2>&1 || exit $?
done
