#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04d
tools/pmc_probe.sh $GRAFT_REPO_ROOT/gpurun_out/r04d/pmc_fresh --fresh || exit $?
python tools/pmc_summary.py gpurun_out/r04d/pmc_fresh config2-fresh gpurun_out/r04d/pmc_fresh_summary.json 2 || exit $?
tools/pmc_probe.sh $GRAFT_REPO_ROOT/gpurun_out/r04d/pmc_fixed || exit $?
python tools/pmc_summary.py gpurun_out/r04d/pmc_fixed config2-fixed gpurun_out/r04d/pmc_fixed_summary.json 2 || exit $?
tools/ab_pool.sh 2 base pipe base@LIVO_XCD_CHUNK=8 || exit $?
