#!/bin/bash
# round 4: the wave-parallel cell walk (walk_wave): parity, the pool's per-batch first evaluations, A/B, side legs
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04k
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ikd_incr.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r04k/pytest_parity_incr.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_mode.py tests/test_gpu_ikfom.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r04k/pytest_bench_ikfom.log 2>&1 || exit $?
timeout -k 10 300 python tools/pool_probe.py --batches 8 > gpurun_out/r04k/pool_probe.txt 2>&1 || exit $?
tools/ab_pool.sh 2 base base@LIVO_XCD_CHUNK=2 base@LIVO_XCD_CHUNK=8 || exit $?
timeout -k 10 300 python bench.py --legs config5,ikd,ikfom --cpu-seconds 0 --pmc off --steps 8 > gpurun_out/r04k/bench_legs.log 2>&1 || exit $?
