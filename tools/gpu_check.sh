#!/bin/bash
# One GPU-box pass: smoke, GPU parity tests, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; steps are chained with && so the
# first failure ends the call.  Logs land in gpurun_out/ (merged back).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-run}"
mkdir -p "$OUT"
cd "$ROOT"
echo "start $(date)" > "$OUT/status.txt"
rocm-smi --showproductname > "$OUT/rocm_smi.txt" 2>&1 || true
lscpu | grep -E "Model name|Socket|^CPU\(s\)" > "$OUT/lscpu.txt" 2>&1 || true
timeout -k 10 600 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && echo "smoke ok" >> "$OUT/status.txt" && \
timeout -k 10 1200 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1 && echo "pytest ok" >> "$OUT/status.txt" && \
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err" && echo "bench ok" >> "$OUT/status.txt" && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof" -o kt --output-format csv -- python3 "$ROOT/bench.py" --no-cpu-baseline --steps 50 > "$OUT/prof.log" 2>&1 && echo "prof ok" >> "$OUT/status.txt"
rc=$?
echo "end rc=$rc $(date)" >> "$OUT/status.txt"
exit $rc
