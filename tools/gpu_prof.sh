#!/bin/bash
# bench + rocprofv3 kernel stats + two PMC passes (FETCH_SIZE, WRITE_SIZE:
# they cannot share a pass on gfx950).  Counters run with --kernel-trace only.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-prof}"
mkdir -p "$OUT"
cd "$ROOT"
echo "start $(date)" > "$OUT/status.txt"
BA="${BENCH_ARGS:-}"
timeout -k 10 600 python bench.py $BA > "$OUT/bench.json" 2> "$OUT/bench.err" && echo "bench ok" >> "$OUT/status.txt" && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o kt --output-format csv -- python3 "$ROOT/bench.py" --no-cpu-baseline $BA > "$OUT/prof.log" 2>&1 && echo "stats ok" >> "$OUT/status.txt" && \
timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o pmc --output-format csv -- python3 "$ROOT/bench.py" --no-cpu-baseline --steps 10 --warmup 2 $BA > "$OUT/pmc_fetch.log" 2>&1 && echo "pmc fetch ok" >> "$OUT/status.txt" && \
timeout -k 10 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/pmc_write" -o pmc --output-format csv -- python3 "$ROOT/bench.py" --no-cpu-baseline --steps 10 --warmup 2 $BA > "$OUT/pmc_write.log" 2>&1 && echo "pmc write ok" >> "$OUT/status.txt"
rc=$?
echo "end rc=$rc $(date)" >> "$OUT/status.txt"
exit $rc
