#!/bin/bash
# round 4: bench-mode GPU tests (new submit / pool-seed cases), the pooled headline, search statistics
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04b
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench_mode.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r04b/pytest_bench_mode.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --legs headline,latency --cpu-seconds 0 --pmc off > gpurun_out/r04b/bench_pool.log 2>&1 || exit $?
LIVO_LIB=fast-livo-noted_amd/lib/variants/evprof.so timeout -k 10 200 python tools/eval_prof.py > gpurun_out/r04b/evprof_c2.txt 2>&1 || exit $?
LIVO_LIB=fast-livo-noted_amd/lib/variants/evprof.so timeout -k 10 300 python tools/eval_prof.py --config5 > gpurun_out/r04b/evprof_c5.txt 2>&1 || exit $?
