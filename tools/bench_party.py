"""Party-side kernels, device-resident: K_CONV, K_ODO_PRE, open, K_ODO_POST,
and the fused open + K_ODO_POST the service runs (k_open_post).

    python tools/bench_party.py [--words W] [--parties N] [--reps R]

Prints one JSON line with each kernel's median duration (HIP events stamped
by the kernel dispatch, amph_time_next_launch) and its algorithmic GB/s
(DESIGN.md §4 bytes per word).  Inputs: uniform random field words
(synthetic; the arithmetic does not depend on their distribution).
"""
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
print(json.dumps(out))
