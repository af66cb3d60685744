#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04iv
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04iv/kt -o kt -- \
    python3 $R/bench.py --legs ivox --steps 5 --cpu-seconds 0 --pmc off > $R/gpurun_out/r04iv/bench.log 2>&1 || exit $?
