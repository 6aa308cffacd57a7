#!/bin/bash
# Rehearsals of the multi-rank code paths on a one-GPU box + C4 scatter mode at world 1.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-multi}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 \
  bench.py --gpus 2 --backend gloo --same-device --steps 20 --no-cpu-baseline > "$OUT/gloo2.json" 2> "$OUT/gloo2.err" && echo "gloo2 ok" >> "$OUT/status.txt" && \
timeout -k 10 300 python bench.py --scatter --words 67108864 --parties 2 --steps 5 --warmup 1 > "$OUT/scatter1.json" 2> "$OUT/scatter1.err" && echo "scatter1 ok" >> "$OUT/status.txt" && \
timeout -k 10 300 python bench.py --words 67108864 --parties 2 --steps 10 --no-cpu-baseline > "$OUT/c4_resident1.json" 2> "$OUT/c4_resident1.err" && echo "c4 ok" >> "$OUT/status.txt"
echo "end rc=$?" >> "$OUT/status.txt"
