#!/bin/bash
# rocprofv3 kernel trace of tools/knn_probe.py (the bench's batch, a few steps).
# usage: tools/prof_probe.sh <out_dir>
set -o pipefail
OUT=$1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o kt -- python3 $GRAFT_REPO_ROOT/tools/knn_probe.py --steps 5
