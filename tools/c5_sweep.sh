#!/bin/bash
# Config-5 bench leg under a list of env settings (tuning sweeps).
# usage: tools/c5_sweep.sh "VAR=VAL[,VAR=VAL]" ...   ("base": no setting); output gpurun_out/c5_<spec>.log
for v in "$@"; do
  e=""; [ "$v" != base ] && e=$(echo "$v" | tr ',' ' ')
  env $e timeout -k 10 200 python bench.py --legs config5 --cpu-seconds 0 --pmc off --steps 8 > gpurun_out/c5_$(echo $v | tr '=,' '-+').log 2>&1 || exit 1
done
