"""Host-memory (PCIe-inclusive) wire-to-wire pipelines of one batch (tool;
DESIGN.md "Round 3 in brief"): the same stages as tools/bench_pipeline.py,
but every buffer a Java caller would hand over lives in host memory, as it
does behind the JNI boundary (jni/amphora_jni.c pins Java heap arrays, which
are pageable):

* party Output Delivery: odo_pre -> exchange text (bytes, as a server sends
  it) -> the N-1 partners' texts decoded -> open_post -> base64 of the five
  ODO fields; then the same through a device-resident party session
  (amph_party_begin / _text / _partner / _finish_b64), where only the texts
  and the base64 fields cross PCIe;
* client download / upload straight from the parties' base64 text
  (amph_recombine_verify_b64 / amph_mask_input_b64).

    python tools/bench_pipeline_host.py [--words W] [--parties N] [--reps R] [--pinned]

--pinned registers the caller's input AND output arrays page-locked first
(amph_host_register), as a caller that owns direct buffers would.  Every
output array is allocated and touched once before timing (a JVM zeroes a new
array when it allocates it, so first-touch page faults are not the call's),
and the stages call the C ABI directly so no Python copy is timed.
Wall-clock per stage (the host calls are synchronous); medians over reps.
Prints one JSON line.
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
import ctypes as C  # noqa: E402
from amphora_amd._lib import lib as L, _ptr, _AmphOdoB64  # noqa: E402
from amphora_amd.spdz import TEST_PRIME, TEST_R, TEST_RINV  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--words", type=int, default=1 << 22)
ap.add_argument("--parties", type=int, default=3)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--pinned", action="store_true")
a = ap.parse_args()
W, n = a.words, a.parties
ctx = A.Context(TEST_PRIME, TEST_R, TEST_RINV)

share = ctx.synth_words(1, 2 * W).view(W, 32).cpu().numpy()
masks = ctx.synth_words(2, 4 * W).view(2 * W, 32).cpu().numpy()
triples = ctx.synth_words(3, 12 * W).view(2 * W, 96).cpu().numpy()
odos, _, _ = ctx.synth_odos(seed=4, n=n, words=W)
mask_odos, _, _ = ctx.synth_odos(seed=5, n=n, words=W)
secrets = ctx.synth_words(6, W).cpu().numpy()
b64_odos = [[bytes(ctx.base64_encode(f.reshape(-1)).cpu().numpy()) for f in o] for o in odos]
b64_masks = [[bytes(ctx.base64_encode(f.reshape(-1)).cpu().numpy()) for f in o] for o in mask_odos]
torch.cuda.synchronize()
b64_odos = [[np.frombuffer(t, np.uint8).copy() for t in o] for o in b64_odos]
b64_masks = [[np.frombuffer(t, np.uint8).copy() for t in o] for o in b64_masks]
h = ctx._h
P = 2 * W  # FactorPairs
y, r, v, w, u = (np.zeros((W, 16), np.uint8) for _ in range(5))
mags = [np.zeros((P, 2, 16), np.uint8) for _ in range(n)]
negs = [np.zeros((P, 2), np.uint8) for _ in range(n)]
cap = L.amph_exchange_max_chars(P)
text = np.zeros(cap, np.uint8)
b64_out = [np.zeros(4 * ((16 * W + 2) // 3), np.uint8) for _ in range(5)]
secrets_out = np.zeros((W, 16), np.uint8)
records = np.zeros((W, 24), np.uint8)
outputs = [y, r, v, w, u, text, secrets_out, records] + mags + negs + b64_out
if a.pinned:
    for x in [share, masks, triples, secrets] + [t for o in b64_odos + b64_masks for t in o] + outputs:
        ctx.host_register(x)
tlen = C.c_uint64(0)
bad = C.c_int64(-1)
ff = C.c_int64(-1)
pm = (C.c_void_p * n)(*[_ptr(m) for m in mags])
pn = (C.c_void_p * n)(*[_ptr(g) for g in negs])


def odo_texts(texts):
    arr = (_AmphOdoB64 * n)()
    for j, t in enumerate(texts):
        arr[j] = _AmphOdoB64(*[_ptr(f) for f in t], t[0].size)
    return arr


b64_odo_arr, b64_mask_arr = odo_texts(b64_odos), odo_texts(b64_masks)


def ok(st):
    if st != 0:
        raise RuntimeError("status %d: %s" % (st, L.amph_last_error().decode()))


def stages(fn):
    per = {}
    for r in range(a.reps + 1):
        marks = [("start", time.perf_counter())]
        fn(lambda name: marks.append((name, time.perf_counter())))
        if r >= 1:
            for (_, t0), (name, t1) in zip(marks, marks[1:]):
                per.setdefault(name, []).append((t1 - t0) * 1e3)
    med = {k: statistics.median(v) for k, v in per.items()}
    tot = sum(med.values())
    return {"stages_ms": {k: round(v, 3) for k, v in med.items()}, "total_ms": round(tot, 3),
            "words_per_s": W / (tot * 1e-3)}


def party(mark):
    ok(L.amph_odo_pre(h, _ptr(share), 32, _ptr(masks), _ptr(triples), W, _ptr(y), _ptr(r), _ptr(v),
                      _ptr(mags[0]), _ptr(negs[0]), 0, None))
    mark("odo_pre")
    ok(L.amph_exchange_encode(h, _ptr(mags[0]), _ptr(negs[0]), P, _ptr(text), cap, C.addressof(tlen), 0, None))
    mark("exchange_encode")
    for j in range(1, n):  # the partners' texts: stand-ins of the same size, this party's own
        ok(L.amph_exchange_decode(h, _ptr(text), tlen.value, P, _ptr(mags[j]), _ptr(negs[j]), C.byref(bad), 0,
                                  None))
    mark("exchange_decode_x%d" % (n - 1))
    ok(L.amph_open_post(h, pm, pn, n, _ptr(triples), W, 0, _ptr(w), _ptr(u), 0, None))
    mark("open_post")
    for f, o in zip((y, r, v, w, u), b64_out):
        ok(L.amph_base64_encode(h, _ptr(f), f.size, _ptr(o), 0, None))
    mark("base64_encode_x5")


def party_session(mark):
    """the same party through amph_party_*: only the texts and the base64 ODO
    fields cross PCIe (y/r/v come back as base64 from finish)"""
    ph = C.c_void_p()
    ok(L.amph_party_begin(h, _ptr(share), 32, _ptr(masks), _ptr(triples), W, n, None, None, None, C.byref(ph)))
    mark("begin")
    ln = L.amph_party_text_len(ph)
    ok(L.amph_party_text(ph, _ptr(text), cap))
    mark("own_text")
    for j in range(1, n):
        ok(L.amph_party_partner(ph, j, _ptr(text), ln, C.byref(bad)))
    mark("partners_x%d" % (n - 1))
    ok(L.amph_party_finish_b64(ph, 0, b64_arr))
    mark("finish_b64")
    L.amph_party_free(ph)


b64_arr = (C.c_void_p * 5)(*[_ptr(o) for o in b64_out])


def download(mark):
    ok(L.amph_recombine_verify_b64(h, b64_odo_arr, n, W, _ptr(secrets_out), C.byref(ff), C.byref(bad), 0, None))
    mark("recombine_verify_b64")


def upload(mark):
    ok(L.amph_mask_input_b64(h, b64_mask_arr, n, W, _ptr(secrets), W, None, _ptr(records), C.byref(ff),
                             C.byref(bad), 0, None))
    mark("mask_input_b64")


out = {"words": W, "parties": n, "memory": "host, page-locked" if a.pinned else "host, pageable",
       "party_output_delivery": stages(party), "party_output_delivery_session": stages(party_session),
       "client_download": stages(download),
       "client_upload": stages(upload),
       "text_bytes": {"exchange": tlen.value, "odo_field_b64": int(b64_odos[0][0].size)}}
print(json.dumps(out))
