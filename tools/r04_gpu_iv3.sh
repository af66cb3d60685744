#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04iv3
timeout -k 10 400 python -u -m pytest tests/test_gpu_ivox.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04iv3/pytest_ivox.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --legs ivox --steps 10 --cpu-seconds 0 --pmc off > gpurun_out/r04iv3/bench.log 2>&1 || exit $?
