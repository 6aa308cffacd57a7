"""Device-resident wire-to-wire pipelines of one batch (tool):

* party Output Delivery (OutputDeliveryService.computeOutputDeliveryObject,
  OutputDeliveryService.java:75-286, + the VerifiableSecretShare response):
  K_ODO_PRE -> own MultiplicationExchangeObject array text (exchange encode)
  -> the N-1 partners' texts parsed (exchange decode) -> open + K_ODO_POST
  (k_open_post) -> base64 of the five ODO fields; once through the per-call
  device API (pair-order decode) and once as a device-mode party session
  (amph_party_*_dev: one-read span-form decode);
* client download (DefaultAmphoraClient.getSecret, :206-217): base64 decode of
  the N parties' five ODO fields -> K_RV;
* client upload (createSecret, :150-170): base64 decode of the N mask ODOs ->
  K_MASK -> base64 of each masked word (the MaskedInput records);
* the same two client paths as ONE launch each from the wire text
  (amph_recombine_verify_b64 / amph_mask_input_b64, *_fused).

    python tools/bench_pipeline.py [--words W] [--parties N] [--reps R]

Every stage runs on the GPU on torch's current stream; the only host
round trip is the exchange text's length (read back once, as a server would
to send it).  Partners' texts are stand-ins: this party's own text parsed
N-1 times (same size and digit distribution).  Prints one JSON line.
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import amphora_amd as A  # noqa: E402
from amphora_amd.spdz import TEST_PRIME, TEST_R, TEST_RINV  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--words", type=int, default=1 << 22)
ap.add_argument("--parties", type=int, default=3)
ap.add_argument("--reps", type=int, default=10)
a = ap.parse_args()
W, n = a.words, a.parties
ctx = A.Context(TEST_PRIME, TEST_R, TEST_RINV)

share = ctx.synth_words(1, 2 * W).view(W, 32)
masks = ctx.synth_words(2, 4 * W).view(2 * W, 32)
triples = ctx.synth_words(3, 12 * W).view(2 * W, 96)
odos, _, _ = ctx.synth_odos(seed=4, n=n, words=W)
mask_odos, _, _ = ctx.synth_odos(seed=5, n=n, words=W)
secrets = ctx.synth_words(6, W)
# the parties' base64 field texts (what the client receives), made on the GPU
b64_odos = [[ctx.base64_encode(f.reshape(-1)) for f in o] for o in odos]
b64_masks = [[ctx.base64_encode(f.reshape(-1)) for f in o] for o in mask_odos]
torch.cuda.synchronize()


def stages(fn):
    """Runs fn(mark) reps times; mark(name) records an event after a stage."""
    per = {}
    for r in range(a.reps + 2):
        evs = [("start", torch.cuda.Event(enable_timing=True))]
        evs[0][1].record()

        def mark(name):
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            evs.append((name, e))
        fn(mark)
        torch.cuda.synchronize()
        if r >= 2:
            for (_, e0), (name, e1) in zip(evs, evs[1:]):
                per.setdefault(name, []).append(e0.elapsed_time(e1))
    med = {k: statistics.median(v) for k, v in per.items()}
    return {"stages_ms": {k: round(v, 4) for k, v in med.items()}, "total_ms": round(sum(med.values()), 4),
            "words_per_s": W / (sum(med.values()) * 1e-3)}


def party(mark):
    y, r, v, mag, neg = ctx.odo_pre(share, 32, masks, triples)
    mark("k_odo_pre")
    text, ln = ctx.exchange_encode(mag, neg)
    L = int(ln.item())  # the body length a server needs to send it
    mark("exchange_encode")
    mags, negs = [mag], [neg]
    for _ in range(n - 1):
        m2, n2, bad = ctx.exchange_decode(text[:L], 2 * W)
        mags.append(m2)
        negs.append(n2)
    mark("exchange_decode_x%d" % (n - 1))
    w, u = ctx.open_post(mags, negs, triples, False)
    mark("k_open_post")
    for f in (y, r, v, w, u):
        ctx.base64_encode(f.reshape(-1))
    mark("base64_encode_x5")


def party_session(mark):
    """The same Output Delivery as a device-mode party session
    (amph_party_*_dev): partner texts decoded in one read into span form,
    finish reading them through the span bases."""
    s = ctx.party_begin_dev(share, 32, masks, triples, n)
    mark("begin (k_odo_pre + encode)")
    t, ln = s.text_dev()
    L = int(ln.item())  # the body length a server needs to send it
    mark("text length read back")
    for slot in range(1, n):
        s.partner(slot, t[:L])
    mark("partners x%d (decode to span form)" % (n - 1))
    s.finish_b64(False)
    mark("finish_b64 (k_open_post + base64 x5)")
    s.close()


def download(mark):
    fields = [tuple(ctx.base64_decode(t, 16 * W)[0].view(W, 16) for t in o) for o in b64_odos]
    mark("base64_decode_x%d" % (5 * n))
    ctx.recombine_verify(fields)
    mark("k_rv")


def upload(mark):
    fields = [tuple(ctx.base64_decode(t, 16 * W)[0].view(W, 16) for t in o) for o in b64_masks]
    mark("base64_decode_x%d" % (5 * n))
    masked, _ = ctx.mask_input(fields, secrets)
    mark("k_mask")
    ctx.base64_encode_words(masked)
    mark("base64_words")


def download_fused(mark):
    ctx.recombine_verify_b64(b64_odos, W)
    mark("k_rv_b64")


def upload_fused(mark):
    ctx.mask_input_b64(b64_masks, W, secrets, records=True)
    mark("k_mask_b64")


out = {"words": W, "parties": n, "party_output_delivery": stages(party),
       "party_output_delivery_session": stages(party_session),
       "client_download": stages(download), "client_upload": stages(upload),
       "client_download_fused": stages(download_fused), "client_upload_fused": stages(upload_fused)}
print(json.dumps(out))
