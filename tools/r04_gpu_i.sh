#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04i
timeout -k 10 600 python -u -m pytest tests/test_gpu_ikd_incr.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r04i/pytest_ikd_incr.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --legs ikd --cpu-seconds 0 --pmc off --steps 8 > gpurun_out/r04i/bench_ikd.log 2>&1 || exit $?
timeout -k 10 300 python tools/pool_probe.py --batches 8 > gpurun_out/r04i/pool_probe.txt 2>&1 || exit $?
LIVO_XCD_CHUNK=8 timeout -k 10 300 python tools/pool_probe.py --batches 8 > gpurun_out/r04i/pool_probe_x8.txt 2>&1 || exit $?
for s0 in 0 24 48; do
  LIVO_LIB=fast-livo-noted_amd/lib/variants/evprof.so timeout -k 10 200 python tools/eval_prof.py --seed0 $s0 > gpurun_out/r04i/evprof_seed$s0.txt 2>&1 || exit $?
done
tools/ab_pool.sh 1 base base@LIVO_XCD_CHUNK=-1 base@LIVO_XCD_CHUNK=1 base@LIVO_XCD_CHUNK=2 base@LIVO_XCD_CHUNK=4 base@LIVO_XCD_CHUNK=8 base@LIVO_XCD_CHUNK=16 base@LIVO_SYNC_ZC=1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_ikfom.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r04i/pytest_ikfom.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --legs ikfom --cpu-seconds 0 --pmc off --steps 10 > gpurun_out/r04i/bench_ikfom.log 2>&1 || exit $?
