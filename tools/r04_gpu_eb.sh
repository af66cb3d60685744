#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
tools/ab_pool.sh 2 base eb128 ew5 || exit $?
