#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04t
LIVO_GRAPH=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_mode.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r04t/pytest_bench_mode_graph.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_ikd_incr.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r04t/pytest_ikd_incr.log 2>&1 || exit $?
tools/ab_pool.sh 2 base base@LIVO_GRAPH=1 || exit $?
LIVO_GRAPH=1 timeout -k 10 300 python bench.py --legs headline,latency --cpu-seconds 0 --pmc off > gpurun_out/r04t/bench_graph.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --legs headline,latency --cpu-seconds 0 --pmc off > gpurun_out/r04t/bench_nograph.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --legs ikd --cpu-seconds 0 --pmc off --steps 2 > gpurun_out/r04t/bench_ikd.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_ikfom.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r04t/pytest_ikfom.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --legs ikfom --cpu-seconds 0 --pmc off --steps 10 > gpurun_out/r04t/bench_ikfom.log 2>&1 || exit $?
LIVO_LIB=fast-livo-noted_amd/lib/variants/ikprof.so timeout -k 10 200 python tools/ik_prof.py > gpurun_out/r04t/ik_prof.txt 2>&1 || exit $?
