#!/bin/bash
# Probe-vs-K_MASK comparison through bench.py at C2 (twice) and C3.
set -o pipefail
mkdir -p gpurun_out/${TAG:-r02_probe}
O=gpurun_out/${TAG:-r02_probe}
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c2_a.json 2> $O/err.txt && \
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c2_b.json 2>> $O/err.txt && \
timeout -k 10 300 python bench.py --no-cpu-baseline --words 16777216 --parties 3 --steps 100 > $O/c3.json 2>> $O/err.txt
