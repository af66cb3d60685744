#!/bin/bash
# round-4 final: the whole -m gpu suite and smoke()
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/final/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || exit $?
