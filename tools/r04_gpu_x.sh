#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
tools/ab_pool.sh 2 base base@LIVO_STREAM_GROUPS=1 base@LIVO_STREAM_GROUPS=4 base@LIVO_BR_HA=1.5 base@LIVO_XCD_CHUNK=2 base@LIVO_SYNC_ZC=1 || exit $?
