#!/bin/bash
# Config-5 bench leg for variant libraries (tools/ab_run.sh spec syntax: LIB[@VAR=VAL,...]).
# usage: tools/c5_ab.sh spec ...; output gpurun_out/c5ab_<spec>.log
for spec in "$@"; do
  n=${spec%%@*}; envs=""
  [ "$spec" != "$n" ] && envs=$(echo "${spec#*@}" | tr ',' ' ')
  if [ "$n" = base ]; then lib=""; else lib=fast-livo-noted_amd/lib/variants/$n.so; fi
  env LIVO_LIB=$lib $envs timeout -k 10 200 python bench.py --legs config5 --cpu-seconds 0 --pmc off --steps 8 \
      > gpurun_out/c5ab_$(echo $spec | tr '@=,/' '+-+-').log 2>&1 || exit 1
done
