#!/bin/bash
# One parameterised GPU job (replaces round 4's one-off tools/r04_gpu_*.sh).
# Runs its steps in order on the gpurun box; the first failing step ends the job.
#
# usage: tools/gpu_job.sh TAG STEP [STEP ...]      output: gpurun_out/TAG/
#   tests[=PATHS]         pytest -m gpu over PATHS (default: tests), one process
#   smoke                 __graft_entry__.smoke()
#   bench[=ARGS]          python bench.py ARGS  (default: the full default line)
#   ab=R=SPEC,SPEC..      pooled-headline A/B in R rounds (tools/ab_pool.sh spec syntax)
#   abs=R=SPEC;SPEC..     the same with ';' between specs (a spec may set several VAR=VAL,VAR=VAL)
#   c5ab=SPEC,SPEC..      config-5 leg per variant (tools/c5_ab.sh)
#   kt[=ARGS]             rocprofv3 --kernel-trace --stats over bench.py ARGS
#                         (default: the headline leg, 20 steps)
#   ktpy=SCRIPT ARGS      rocprofv3 --kernel-trace --stats over python3 SCRIPT ARGS (repo-relative script)
#   ktcp=SCRIPT ARGS      the same with --memory-copy-trace (copy durations)
#   pmc_eval              PMC passes over the first evaluation (tools/pmc_eval.sh)
#   pmc_c5                PMC passes over the config-5 batch (tools/pmc_c5.sh)
#   py=SCRIPT ARGS        python SCRIPT ARGS (any lab/probe script), 200 s limit
#   env=VAR=VAL,..        export for the steps that follow
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=$1; shift
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
n=0
for step in "$@"; do
  n=$((n+1))
  kind=${step%%=*}
  arg=""; [ "$step" != "$kind" ] && arg=${step#*=}
  log=$OUT/$(printf %02d $n)_$kind.log
  echo "[gpu_job] step $n: $step -> $log"
  case $kind in
    tests)
      timeout -k 10 1100 python -u -m pytest ${arg:-tests} -m gpu -x -v --timeout 300 --timeout-method thread \
          > "$log" 2>&1 || { tail -30 "$log"; exit 1; } ;;
    smoke)
      timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > "$log" 2>&1 || { tail -30 "$log"; exit 1; } ;;
    bench)
      timeout -k 10 700 python bench.py $arg > "$log" 2> "$log.err" || { tail -30 "$log.err"; exit 1; }
      tail -1 "$log" ;;
    ab)
      rounds=${arg%%=*}; specs=$(echo "${arg#*=}" | tr ',' ' ')
      (cd "$R" && bash tools/ab_pool.sh "$rounds" $specs) > "$log" 2>&1 || { tail -30 "$log"; exit 1; }
      python tools/ab_summary.py gpurun_out >> "$log" 2>&1; tail -20 "$log" ;;
    abs)  # as ab, specs separated by ';' so a spec can carry several VAR=VAL (comma-separated)
      rounds=${arg%%=*}; specs=$(echo "${arg#*=}" | tr ';' ' ')
      (cd "$R" && bash tools/ab_pool.sh "$rounds" $specs) > "$log" 2>&1 || { tail -30 "$log"; exit 1; }
      python tools/ab_summary.py gpurun_out >> "$log" 2>&1; tail -20 "$log" ;;
    c5ab)
      bash tools/c5_ab.sh $(echo "$arg" | tr ',' ' ') > "$log" 2>&1 || { tail -30 "$log"; exit 1; } ;;
    kt)
      a=${arg:-"--legs headline --steps 20 --warmup 3 --cpu-seconds 0 --pmc off"}
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$OUT/kt$n" -o kt -- python3 "$R/bench.py" $a) > "$log" 2>&1 || { tail -30 "$log"; exit 1; } ;;
    ktpy)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$OUT/kt$n" -o kt -- python3 $(echo "$arg" | sed "s|^|$R/|")) > "$log" 2>&1 || { tail -30 "$log"; exit 1; } ;;
    ktcp)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats \
          --output-format csv -d "$OUT/kt$n" -o kt -- python3 $(echo "$arg" | sed "s|^|$R/|")) > "$log" 2>&1 || { tail -30 "$log"; exit 1; } ;;
    pmc_eval)
      bash tools/pmc_eval.sh "$OUT/pmc$n" > "$log" 2>&1 || { tail -30 "$log"; exit 1; } ;;
    pmc_c5)
      bash tools/pmc_c5.sh "$OUT/pmc$n" > "$log" 2>&1 || { tail -30 "$log"; exit 1; }
      python tools/pmc_summary.py "$OUT/pmc$n" config5 "$OUT/c5pmc_summary.json" 4 >> "$log" 2>&1 ;;
    py)
      timeout -k 10 200 python $arg > "$log" 2>&1 || { tail -30 "$log"; exit 1; }
      tail -5 "$log" ;;
    env)
      for kv in $(echo "$arg" | tr ',' ' '); do export "$kv"; done ;;
    *)
      echo "[gpu_job] unknown step $step"; exit 2 ;;
  esac
done
echo "[gpu_job] done"
