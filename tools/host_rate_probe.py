"""Host-path rate probe (tool): pageable host calls of the batched pipeline
(odo_pre, open_post, mask_input) at 4 Mi words x 3 parties with different
staging-thread counts (AMPH_HOST_THREADS) and batch sizes (amph_ctx_set_batch_words),
beside plain blocking pageable hipMemcpy (torch .cuda() / .cpu()) of the same
byte counts.  Outputs go to caller buffers allocated once (out=).  Prints JSON lines.

    python tools/host_rate_probe.py [--words W] [--threads 8] [--batches 4194304,1048576,524288]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import amphora_amd as A  # noqa: E402
from amphora_amd.spdz import TEST_PRIME, TEST_R, TEST_RINV  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--words", type=int, default=1 << 22)
ap.add_argument("--threads", default="8")
ap.add_argument("--batches", default="4194304,1048576,524288,262144")
ap.add_argument("--reps", type=int, default=4)
a = ap.parse_args()
W, n = a.words, 3


def med(fn):
    ts = []
    for r in range(a.reps + 1):
        t0 = time.perf_counter()
        fn()
        if r:
            ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


# raw pageable copies
for gb in (1,):
    host = np.ones(gb << 30, np.uint8)
    dev = torch.empty(gb << 30, dtype=torch.uint8, device="cuda")
    back = np.empty_like(host)
    th = torch.from_numpy(host)
    tb = torch.from_numpy(back)
    h2d = med(lambda: (dev.copy_(th), torch.cuda.synchronize()))
    d2h = med(lambda: (tb.copy_(dev), torch.cuda.synchronize()))
    print(json.dumps({"probe": "pageable torch copy", "bytes": host.nbytes, "h2d_GBps": host.nbytes / h2d / 1e9,
                      "d2h_GBps": host.nbytes / d2h / 1e9}), flush=True)
    del host, dev, back, th, tb

ctx0 = A.Context(TEST_PRIME, TEST_R, TEST_RINV)
share = ctx0.synth_words(1, 2 * W).view(W, 32).cpu().numpy()
masks = ctx0.synth_words(2, 4 * W).view(2 * W, 32).cpu().numpy()
triples = ctx0.synth_words(3, 12 * W).view(2 * W, 96).cpu().numpy()
odos_d, _, _ = ctx0.synth_odos(seed=4, n=n, words=W)
odos = [tuple(f.cpu().numpy() for f in o) for o in odos_d]
secrets = ctx0.synth_words(6, W).cpu().numpy()
y, r, v, mag, neg = ctx0.odo_pre(share, 32, masks, triples)
mags, negs = [mag] * n, [neg] * n
out = np.zeros((W, 16), np.uint8)
L, P_ = A._lib.lib, A._lib._ptr
yo, ro, vo, wo, uo = (np.zeros((W, 16), np.uint8) for _ in range(5))
mo, no = np.zeros((2 * W, 2, 16), np.uint8), np.zeros((2 * W, 2), np.uint8)
import ctypes as C  # noqa: E402
pm = (C.c_void_p * n)(*[P_(m) for m in mags])
pn = (C.c_void_p * n)(*[P_(g) for g in negs])


def pre_call(ctx):
    A.Context._check(L.amph_odo_pre(ctx._h, P_(share), 32, P_(masks), P_(triples), W, P_(yo), P_(ro), P_(vo),
                                    P_(mo), P_(no), 0, None))


def post_call(ctx):
    A.Context._check(L.amph_open_post(ctx._h, pm, pn, n, P_(triples), W, 0, P_(wo), P_(uo), 0, None))


for t, bw in [(int(t), int(b)) for t in a.threads.split(",") for b in a.batches.split(",")]:
    os.environ["AMPH_HOST_THREADS"] = str(t)
    ctx = A.Context(TEST_PRIME, TEST_R, TEST_RINV)  # its copy pool reads AMPH_HOST_THREADS
    ctx.set_batch_words(bw)
    t_pre = med(lambda: pre_call(ctx))
    t_post = med(lambda: post_call(ctx))
    t_mask = med(lambda: ctx.mask_input(odos, secrets, out=out))
    b_pre = W * (32 + 64 + 192 + 48 + 68)
    b_post = W * (n * 68 + 192 + 32)
    b_mask = W * (80 * n + 16 + 16)
    print(json.dumps({"probe": "batched host calls, pageable", "words": W, "parties": n, "host_threads": t, "batch_words": bw,
                      "odo_pre_ms": t_pre * 1e3, "odo_pre_GBps": b_pre / t_pre / 1e9,
                      "open_post_ms": t_post * 1e3, "open_post_GBps": b_post / t_post / 1e9,
                      "mask_input_ms": t_mask * 1e3, "mask_input_GBps": b_mask / t_mask / 1e9}), flush=True)
    del ctx
