#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04s
timeout -k 10 400 python -u -m pytest tests/test_gpu_ikfom.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r04s/pytest_ikfom.log 2>&1 || exit $?
LIVO_LIB=fast-livo-noted_amd/lib/variants/ikprof.so timeout -k 10 200 python tools/ik_prof.py > gpurun_out/r04s/ik_prof.txt 2>&1 || exit $?
timeout -k 10 200 python bench.py --legs ikfom --cpu-seconds 0 --pmc off --steps 10 > gpurun_out/r04s/bench_ikfom.log 2>&1 || exit $?
for m in 4096 1000000000; do
  LIVO_DYN_DRUNS_MIN=$m timeout -k 10 300 python bench.py --legs ikd --cpu-seconds 0 --pmc off --steps 2 > gpurun_out/r04s/ikd_drmin_$m.log 2>&1 || exit $?
done
