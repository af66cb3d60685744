#!/bin/bash
# round 4: index runs — parity tests first, then pooled A/B and the per-batch pool probe
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04f
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r04f/pytest_parity.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_mode.py -x -v --timeout 300 --timeout-method thread -k "headline or golden" \
    > gpurun_out/r04f/pytest_bench_mode.log 2>&1 || exit $?
tools/ab_pool.sh 2 base f4runs base@LIVO_XCD_CHUNK=8 || exit $?
timeout -k 10 300 python tools/pool_probe.py --batches 12 > gpurun_out/r04f/pool_probe_idx.txt 2>&1 || exit $?
LIVO_LIB=fast-livo-noted_amd/lib/variants/f4runs.so timeout -k 10 300 python tools/pool_probe.py --batches 12 > gpurun_out/r04f/pool_probe_f4.txt 2>&1 || exit $?
