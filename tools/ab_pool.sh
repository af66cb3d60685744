#!/bin/bash
# Pooled-headline A/B (bench.py --legs headline on distinct scans) over env variants, in rounds.
# usage: tools/ab_pool.sh ROUNDS spec ...   spec = LIB[@VAR=VAL,...] as tools/ab_run.sh
set -o pipefail
R=$1; shift
for r in $(seq 1 $R); do
  for spec in "$@"; do
    n=${spec%%@*}; envs=""
    [ "$spec" != "$n" ] && envs=$(echo "${spec#*@}" | tr ',' ' ')
    if [ "$n" = base ]; then lib=""; else lib=fast-livo-noted_amd/lib/variants/$n.so; fi
    tag=$(echo "$spec" | tr '@=,/' '+-+-')
    env LIVO_LIB=$lib $envs timeout -k 10 200 python bench.py --steps 20 --warmup 3 --cpu-seconds 0 \
        --legs headline --pmc off > gpurun_out/ab_${tag}_$r.log 2>&1 || exit $?
  done
done
