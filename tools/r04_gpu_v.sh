#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04v
for s0 in 0 24 48; do
  LIVO_LIB=fast-livo-noted_amd/lib/variants/evprof.so LIVO_STREAM_GROUPS=1 timeout -k 10 200 python tools/eval_timeline.py --seed0 $s0 --top > gpurun_out/r04v/tl_seed$s0.txt 2>&1 || exit $?
done
timeout -k 10 200 python -u -m pytest tests/test_gpu_ivox.py -k eviction_runs -s -q > gpurun_out/r04v/ivox_passes.txt 2>&1 || exit $?
tools/ab_pool.sh 2 base base@LIVO_BR_R=4.5 base@LIVO_BR_R=6 || exit $?
for r in 3.2 4.5 6; do
  LIVO_BR_R=$r timeout -k 10 300 python bench.py --legs config5 --steps 8 --cpu-seconds 0 --pmc off > gpurun_out/r04v/c5_r$r.log 2>&1 || exit $?
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_ikfom.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04v/pytest_ikfom.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --legs ikfom --cpu-seconds 0 --pmc off --steps 10 > gpurun_out/r04v/bench_ikfom.log 2>&1 || exit $?
LIVO_LIB=fast-livo-noted_amd/lib/variants/ikprof.so timeout -k 10 200 python tools/ik_prof.py > gpurun_out/r04v/ik_prof.txt 2>&1 || exit $?
