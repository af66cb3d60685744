#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04h
timeout -k 10 600 python -u -m pytest tests/test_gpu_ikd_incr.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r04h/pytest_ikd_incr.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --legs ikd --cpu-seconds 0 --pmc off --steps 8 > gpurun_out/r04h/bench_ikd.log 2>&1 || exit $?
timeout -k 10 300 python tools/pool_probe.py --batches 8 > gpurun_out/r04h/pool_probe.txt 2>&1 || exit $?
for s0 in 0 24 48; do
  LIVO_LIB=fast-livo-noted_amd/lib/variants/evprof.so timeout -k 10 200 python tools/eval_prof.py --seed0 $s0 > gpurun_out/r04h/evprof_seed$s0.txt 2>&1 || exit $?
done
