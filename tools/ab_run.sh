#!/bin/bash
# A/B of variant libraries on one box: bench headline leg (no CPU baseline, no
# PMC) for each variant, repeated in rounds so box drift hits all alike.
# usage: tools/ab_run.sh ROUNDS spec1 spec2 ...
#   spec = LIB[@VAR=VAL,VAR=VAL]   LIB "base" = the regular library, else
#          fast-livo-noted_amd/lib/variants/LIB.so; the env assignments apply to that run
# output: gpurun_out/ab_<spec>_<round>.log
set -o pipefail
R=$1; shift
for r in $(seq 1 $R); do
  for spec in "$@"; do
    n=${spec%%@*}
    envs=""
    [ "$spec" != "$n" ] && envs=$(echo "${spec#*@}" | tr ',' ' ')
    if [ "$n" = base ]; then lib=""; else lib=fast-livo-noted_amd/lib/variants/$n.so; fi
    tag=$(echo "$spec" | tr '@=,/' '+-+-')
    env LIVO_LIB=$lib $envs timeout -k 10 120 python bench.py --steps 40 --warmup 10 --cpu-seconds 0 \
        --legs headline --pmc off > gpurun_out/ab_${tag}_$r.log 2>&1 || exit $?
  done
done
