#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04p
timeout -k 10 400 python -u -m pytest tests/test_gpu_ivox.py -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/r04p/pytest_ivox.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --legs ikd --cpu-seconds 0 --pmc off --steps 8 > gpurun_out/r04p/bench_ikd.log 2>&1 || exit $?
LIVO_DYN_RUNS=0 timeout -k 10 300 python bench.py --legs ikd --cpu-seconds 0 --pmc off --steps 8 > gpurun_out/r04p/bench_ikd_noruns.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04p/prof_ikfom -o ik --output-format csv -- python3 bench.py --legs ikfom --cpu-seconds 0 --pmc off --steps 5 > gpurun_out/r04p/bench_ikfom_prof.log 2>&1 || exit $?
