#!/bin/bash
# round 4, first GPU call: config-5 PMC capture (base), then run-scan pipelining A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04a
tools/pmc_c5.sh $GRAFT_REPO_ROOT/gpurun_out/r04a/c5pmc || exit $?
python tools/pmc_summary.py gpurun_out/r04a/c5pmc config5 gpurun_out/r04a/c5pmc_summary.json 4 || exit $?
tools/ab_run.sh 2 base pipe || exit $?
tools/c5_ab.sh base pipe || exit $?
