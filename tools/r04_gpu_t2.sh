#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04t2
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "writeback or stream_groups" -x -v --timeout 200 --timeout-method thread > gpurun_out/r04t2/pytest.log 2>&1 || exit $?
