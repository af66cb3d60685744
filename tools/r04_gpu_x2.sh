#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
tools/ab_pool.sh 2 base base@LIVO_BR_HA=1.5 base@LIVO_BR_HA=2.5 base@LIVO_XCD_CHUNK=4 base@LIVO_XCD_CHUNK=16 base@LIVO_LANE_SERIAL=1 || exit $?
