"""Party-side kernels, device-resident: K_CONV, K_ODO_PRE, open, K_ODO_POST,
and the fused open + K_ODO_POST the service runs (k_open_post).

    python tools/bench_party.py [--words W] [--parties N] [--reps R]

Prints one JSON line with each kernel's median duration (HIP events stamped
by the kernel dispatch, amph_time_next_launch) and its algorithmic GB/s
(DESIGN.md §4 bytes per word).  Inputs: uniform random field words
(synthetic; the arithmetic does not depend on their distribution).

`cpu_baseline`: the same rows on the host cores -- the C oracle
(oracle/amphora_oracle.c, the reference's BigInteger algorithm restated with
schoolbook products and Knuth division, OpenMP) on a bounded 65 536-word
sample, each row timed for --cpu-seconds (0 skips it).  The oracle is the
checker, timed here as the CPU stand-in for the service's Java path; the GPU
rows never touch it.
"""
import time
import argparse
import ctypes as C
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import amphora_amd as A  # noqa: E402
from amphora_amd.spdz import TEST_PRIME, TEST_R, TEST_RINV  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--words", type=int, default=1 << 24)
ap.add_argument("--parties", type=int, default=2)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--cpu-seconds", type=float, default=2.0, help="per row; 0 skips the CPU baseline")
ap.add_argument("--cpu-threads", type=int, default=16)
a = ap.parse_args()
W, n = a.words, a.parties
ctx = A.Context(TEST_PRIME, TEST_R, TEST_RINV)
masked = ctx.synth_words(1, W)
tuples = ctx.synth_words(2, 2 * W).view(W, 32)
share = torch.empty((W, 32), dtype=torch.uint8, device="cuda")
masks = ctx.synth_words(3, 4 * W).view(2 * W, 32)
triples = ctx.synth_words(4, 12 * W).view(2 * W, 96)
partner = [(ctx.synth_words(10 + j, 4 * W).view(2 * W, 2, 16),
            (ctx.synth_words(20 + j, W)[:, :4] & 1).contiguous().view(2 * W, 2)) for j in range(n - 1)]
torch.cuda.synchronize()
L = A._lib.lib
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
for e in ev:
    e.record()
torch.cuda.synchronize()


def timed(fn):
    ts = []
    for r in range(a.reps + 3):
        L.amph_time_next_launch(ev[0].cuda_event, ev[1].cuda_event)
        out = fn()
        torch.cuda.synchronize()
        if r >= 3:
            ts.append(ev[0].elapsed_time(ev[1]))
    return statistics.median(ts), out


res = {}
t, _ = timed(lambda: ctx.convert_share(masked, tuples, 12345, False))
res["k_conv"] = (t, 80)
t, pre = timed(lambda: ctx.odo_pre(share, 32, masks, triples))
res["k_odo_pre"] = (t, 32 + 64 + 192 + 48 + 64 + 4)
y, r, v, mag, neg = pre
mags = [mag] + [p[0] for p in partner]
negs = [neg] + [p[1] for p in partner]
t, opened = timed(lambda: ctx.open_diffs(mags, negs))
res["k_open"] = (t, 68 * n + 64)
t, _ = timed(lambda: ctx.odo_post(opened, triples, True))
res["k_odo_post"] = (t, 64 + 192 + 32)
t, _ = timed(lambda: ctx.open_post(mags, negs, triples, True))
res["k_open_post"] = (t, 68 * n + 192 + 32)  # the product path: open + post fused
out = {"words": W, "parties": n,
       "kernels": {k: {"ms": round(t, 4), "bytes_per_word": b,
                       "GBps": round(b * W / (t * 1e-3) / 1e9, 1),
                       "frac_of_8TBps": round(b * W / (t * 1e-3) / 8e12, 3)} for k, (t, b) in res.items()}}


def cpu_baseline(seconds, threads):
    """Words/s of the C oracle per row (rank-0 host cores, bounded sample)."""
    import numpy as np
    from oracle import coracle
    F = coracle.test_field(threads=threads)
    Ws = 1 << 16
    rng = np.random.default_rng(5)
    words = lambda k: F.synth_words(seed=int(rng.integers(1 << 30)), count=k)  # noqa: E731
    masked_h, tuples_h = words(Ws), words(2 * Ws).reshape(Ws, 32)
    share_h, masks_h, triples_h = words(2 * Ws).reshape(Ws, 32), words(4 * Ws).reshape(2 * Ws, 32), \
        words(12 * Ws).reshape(2 * Ws, 96)
    _, _, _, mag_h, neg_h = F.odo_pre(share_h, 32, masks_h, triples_h)
    mags_h = [mag_h] + [words(4 * Ws).reshape(2 * Ws, 2, 16) for _ in range(n - 1)]
    negs_h = [neg_h] + [(rng.integers(0, 2, (2 * Ws, 2))).astype(np.uint8) for _ in range(n - 1)]
    opened_h = F.recombine_diffs(mags_h, negs_h)

    def rate(fn):
        fn()  # warm-up
        done, t0 = 0, time.perf_counter()
        while True:
            fn()
            done += Ws
            el = time.perf_counter() - t0
            if el >= seconds:
                return done / el
    rows = {
        "k_conv": lambda: F.convert_share(masked_h, tuples_h, 12345, False),
        "k_odo_pre": lambda: F.odo_pre(share_h, 32, masks_h, triples_h),
        "k_open": lambda: F.recombine_diffs(mags_h, negs_h),
        "k_odo_post": lambda: F.odo_post(opened_h, triples_h, True),
        "k_open_post": lambda: F.odo_post(F.recombine_diffs(mags_h, negs_h), triples_h, True),
    }
    return {"kind": "port", "cores": F.threads, "sample_words": Ws, "seconds_per_row": seconds,
            "words_per_s": {k: round(rate(fn)) for k, fn in rows.items()},
            "what": "C oracle (schoolbook product + Knuth division per fromGfp/toGfp/multiply, as "
                    "BigInteger does; OpenMP) restating the service's SecretShareUtil / "
                    "OutputDeliveryService arithmetic"}


for k, (t, b) in res.items():
    out["kernels"][k]["words_per_s"] = round(W / (t * 1e-3))
if a.cpu_seconds > 0:
    cb = cpu_baseline(a.cpu_seconds, a.cpu_threads)
    out["cpu_baseline"] = cb
    out["gpu_over_cpu"] = {k: round(out["kernels"][k]["words_per_s"] / v, 1)
                           for k, v in cb["words_per_s"].items()}
print(json.dumps(out))
