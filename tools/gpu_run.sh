#!/bin/bash
# The one GPU runner: a list of steps separated by `::`, each under its own
# time limit, output under gpurun_out/$TAG/<n>_<kind>.*; the first failing
# step ends the call (nothing more touches the GPU after a fault or timeout).
#
#   TAG=r6a tools/gpu_run.sh smoke :: tests :: bench --steps 20 :: stats :: pmc FETCH_SIZE
#
# kinds:
#   smoke                        __graft_entry__.smoke()
#   tests [pytest args]          default: the whole -m gpu suite
#   bench [bench.py args]        one JSON line -> <n>_bench.json
#   stats [bench.py args]        rocprofv3 --kernel-trace --stats of bench.py
#   pmc COUNTERS [bench args]    one rocprofv3 --pmc pass of bench.py (--kernel-trace only beside it)
#   py LIMIT SCRIPT [args]       python -u SCRIPT args
#   statspy SCRIPT [args]        rocprofv3 --kernel-trace --stats of a python script
#   pmcpy COUNTERS SCRIPT [args] one --pmc pass of a python script
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-run}"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
echo "start $(date)" > "$OUT/status.txt"
n=0
run_step() {
  local kind=$1
  shift
  n=$((n + 1))
  local base="$OUT/${n}_$kind" rc
  case "$kind" in
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$base.log" 2>&1 ;;
    tests) if [ $# -eq 0 ]; then set -- -m gpu tests; fi
           timeout -k 10 1500 python -u -m pytest -x -v --timeout 120 --timeout-method thread "$@" > "$base.log" 2>&1 ;;
    bench) timeout -k 10 600 python -u bench.py "$@" > "$base.json" 2> "$base.err" ;;
    stats) timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$base" -o kt --output-format csv -- \
             python3 "$ROOT/bench.py" --no-cpu-baseline "$@" > "$base.log" 2>&1 ;;
    pmc) local c=$1; shift
         timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $c -d "$base" -o pmc --output-format csv -- \
           python3 "$ROOT/bench.py" --no-cpu-baseline "$@" > "$base.log" 2>&1 ;;
    py) local lim=$1; shift
        timeout -k 10 "$lim" python -u "$@" > "$base.log" 2>&1 ;;
    statspy) timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$base" -o kt --output-format csv -- \
               python3 "$@" > "$base.log" 2>&1 ;;
    pmcpy) local c=$1; shift
           timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $c -d "$base" -o pmc --output-format csv -- \
             python3 "$@" > "$base.log" 2>&1 ;;
    *) echo "unknown step kind: $kind" > "$base.log"; false ;;
  esac
  rc=$?
  echo "$n $kind $* rc=$rc $(date +%T)" >> "$OUT/status.txt"
  return $rc
}
args=()
rc=0
for x in "$@" "::"; do
  if [ "$x" = "::" ]; then
    if [ ${#args[@]} -gt 0 ]; then
      run_step "${args[@]}" || { rc=$?; break; }
    fi
    args=()
  else
    args+=("$x")
  fi
done
echo "end rc=$rc $(date)" >> "$OUT/status.txt"
exit $rc
