#!/bin/bash
# One parameterised GPU-box runner (replaces the per-experiment tools/gpu_*.sh scripts).  Every step runs
# under its own time limit, logs under gpurun_out/, prints a one-line verdict, and exits non-zero on failure
# so steps chain with &&:
#
#   tools/gpu.sh tests [PYTEST_PATHS_OR_ARGS...]       pytest -m gpu (default: tests/; XOPT= runs past failures)
#   tools/gpu.sh smoke                                 __graft_entry__.smoke()
#   tools/gpu.sh bench [BENCH_ARGS...]                 bench.py, JSON line -> gpurun_out/bench.json
#   tools/gpu.sh run NAME SECONDS CMD...               any python command, log gpurun_out/NAME.log
#   tools/gpu.sh prof NAME SECONDS CMD...              rocprofv3 --kernel-trace --stats (no counters)
#   tools/gpu.sh pmc NAME "COUNTERS" SECONDS CMD...    rocprofv3 --pmc (one pass; never with trace domains)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out
mkdir -p "$O"
step=$1; shift
case "$step" in
  tests)
    tag=${TAG:-gpu}
    [ $# -eq 0 ] && set -- tests/
    cd "$R" && timeout -k 10 ${LIMIT:-900} python -u -m pytest "$@" ${XOPT--x} -q -m gpu --timeout 120 --timeout-method thread \
      > "$O/pytest_$tag.log" 2>&1 && { echo "TESTS_OK $(tail -1 "$O/pytest_$tag.log")"; } \
      || { tail -40 "$O/pytest_$tag.log"; exit 1; } ;;
  smoke)
    cd "$R" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
      && echo "SMOKE_OK $(tail -1 "$O/smoke.log")" || { tail -30 "$O/smoke.log"; exit 1; } ;;
  bench)
    tag=${TAG:-bench}
    cd "$R" && timeout -k 10 ${LIMIT:-600} python bench.py "$@" > "$O/$tag.log" 2>&1 \
      && { tail -1 "$O/$tag.log" > "$O/$tag.json"; echo BENCH_OK; cat "$O/$tag.json"; } \
      || { tail -30 "$O/$tag.log"; exit 1; } ;;
  run)
    name=$1; secs=$2; shift 2
    cd "$R" && timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1 && { echo "RUN_OK $name"; tail -40 "$O/$name.log"; } \
      || { echo "RUN_FAIL $name"; tail -40 "$O/$name.log"; exit 1; } ;;
  prof)
    name=$1; secs=$2; shift 2
    cd /tmp && timeout -k 10 "$secs" rocprofv3 --kernel-trace --stats -d "$O/prof_$name" -o "$name" -- "$@" \
      > "$O/prof_$name.log" 2>&1 && echo "PROF_OK $name" || { tail -30 "$O/prof_$name.log"; exit 1; }
    # gpurun copies back at most 64 MiB: keep the stats, compress the per-dispatch traces
    find "$O/prof_$name" -name '*.csv' -size +1M -exec gzip -9 {} \; ;;
  pmc)
    name=$1; ctrs=$2; secs=$3; shift 3
    cd /tmp && timeout -s KILL "$secs" rocprofv3 --pmc $ctrs --output-format csv -d "$O/pmc_$name" -o "$name" -- "$@" \
      > "$O/pmc_$name.log" 2>&1 && echo "PMC_OK $name" || { tail -20 "$O/pmc_$name.log"; exit 1; } ;;
  *)
    echo "usage: tools/gpu.sh tests|smoke|bench|run|prof|pmc ..." >&2; exit 2 ;;
esac
