#!/bin/bash
# Fused wire-format kernels: parity tests, then the wire-to-wire pipelines.
set -o pipefail
O=gpurun_out/${TAG:-wire}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_wire_fused.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 200 python tools/bench_pipeline.py --words 4194304 --parties 3 > $O/p3.json 2> $O/err.txt && \
timeout -k 10 200 python tools/bench_pipeline.py --words 1048576 --parties 2 > $O/p2.json 2>> $O/err.txt
