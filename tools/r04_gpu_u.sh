#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04u
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench_mode.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r04u/pytest_wb.log 2>&1 || exit $?
tools/ab_pool.sh 2 base base@LIVO_SLOT_WB=0 || exit $?
timeout -k 10 300 python bench.py --legs headline,latency --cpu-seconds 0 --pmc off > gpurun_out/r04u/bench_wb.log 2>&1 || exit $?
LIVO_SLOT_WB=0 timeout -k 10 300 python bench.py --legs headline,latency --cpu-seconds 0 --pmc off > gpurun_out/r04u/bench_nowb.log 2>&1 || exit $?
