#!/bin/bash
# Parameterised GPU-box recipes (one script instead of per-experiment one-offs).  Every step runs
# under its own time limit through tools/gpu_steps.sh, which stops at the first fatal exit.
#   bash tools/gpu_recipes.sh tests [PYTEST_ARGS...]        pytest -m gpu (or the given tests)
#   bash tools/gpu_recipes.sh bench NAME [BENCH_ARGS...]    bench.py -> gpurun_out/NAME.log
#   bash tools/gpu_recipes.sh prof NAME [BENCH_ARGS...]     rocprofv3 --kernel-trace --stats of bench.py
#   bash tools/gpu_recipes.sh pmc NAME COUNTERS [BENCH_ARGS...]   one PMC pass (own run, no traces)
#   bash tools/gpu_recipes.sh ab NAME VAR "V1 V2 .." [BENCH_ARGS...]  bench once per env value
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
here="$(dirname "$0")"
what="$1"; shift
case "$what" in
  tests)
    args="${*:-tests -m gpu}"
    bash "$here/gpu_steps.sh" gpu_tests 900 \
      "python -u -m pytest -x -v --timeout 240 --timeout-method thread $args" ;;
  bench)
    name="$1"; shift
    bash "$here/gpu_steps.sh" "$name" 400 "python bench.py $*" ;;
  prof)
    name="$1"; shift
    bash "$here/gpu_steps.sh" "$name" 400 \
      "rocprofv3 --kernel-trace --stats -d gpurun_out/$name -o run -- python3 bench.py $*" \
      && python tools/prof_summary.py $(find "gpurun_out/$name" -name '*results.db' | head -1) ${PROF_MARKER:+--marker $PROF_MARKER --skip ${PROF_SKIP:-3}} --steps "${PROF_STEPS:-1}" \
         > "gpurun_out/$name.summary.md" && rm -rf "gpurun_out/$name" ;;  # the database alone can exceed what gpurun copies back
  pmc)
    name="$1"; counters="$2"; shift 2
    bash "$here/gpu_steps.sh" "$name" 120 \
      "timeout -s KILL 100 rocprofv3 --pmc $counters -d gpurun_out/$name -o run -- python3 bench.py $*" ;;
  ab)
    name="$1"; var="$2"; vals="$3"; shift 3
    for v in $vals; do
      bash "$here/gpu_steps.sh" "${name}_$v" 400 "env $var=$v python bench.py $*" || exit $?
    done ;;
  *) echo "unknown recipe $what"; exit 2 ;;
esac
