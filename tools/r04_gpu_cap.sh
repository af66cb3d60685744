#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04cap
for v in base cap64 cap96 base; do
  if [ $v = base ]; then lib=""; else lib=fast-livo-noted_amd/lib/variants/$v.so; fi
  LIVO_LIB=$lib timeout -k 10 300 python bench.py --legs ivox --steps 10 --cpu-seconds 0 --pmc off > gpurun_out/r04cap/$v.log 2>&1 || exit $?
  cp gpurun_out/r04cap/$v.log gpurun_out/r04cap/${v}_$(date +%s).log
done
