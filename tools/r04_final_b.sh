#!/bin/bash
# round-4 final: the default bench line (PMC passes and CPU baseline included),
# a rocprofv3 kernel trace + stats of the headline, PMC passes over the
# first-evaluation kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final
timeout -k 10 600 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || exit $?
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/final/kt -o kt -- \
    python3 $R/bench.py --legs headline --steps 20 --warmup 3 --cpu-seconds 0 --pmc off > $R/gpurun_out/final/kt_bench.log 2>&1 || exit $?
bash $R/tools/pmc_eval.sh $R/gpurun_out/final/pmc > $R/gpurun_out/final/pmc.log 2>&1 || exit $?
