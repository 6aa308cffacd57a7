"""Device-resident throughput of the base64 wire codec kernels (tool).
Bytes counted: input read + output written (algorithmic)."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import amphora_amd as A  # noqa: E402
from amphora_amd.spdz import TEST_PRIME, TEST_R, TEST_RINV  # noqa: E402

ctx = A.Context(TEST_PRIME, TEST_R, TEST_RINV)
L = A._lib.lib
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
for e in ev:
    e.record()
torch.cuda.synchronize()


def timed(fn, reps=20):
    ts = []
    for r in range(reps + 3):
        L.amph_time_next_launch(ev[0].cuda_event, ev[1].cuda_event)
        out = fn()
        torch.cuda.synchronize()
        if r >= 3:
            ts.append(ev[0].elapsed_time(ev[1]))
    return statistics.median(ts), out


n = 3 * (1 << 28)  # 768 MiB of bytes -> 1 GiB of base64
raw = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
t_enc, enc = timed(lambda: ctx.base64_encode(raw))
t_dec, _ = timed(lambda: ctx.base64_decode(enc)[0])  # includes the 2-byte padding read-back
W = 1 << 24
words = ctx.synth_words(1, W)
t_w, rec = timed(lambda: ctx.base64_encode_words(words))
t_uw, _ = timed(lambda: ctx.base64_decode_words(rec)[0])
out = {"stream_bytes": n,
       "b64_encode": {"ms": t_enc, "GBps": (n + 4 * n // 3) / (t_enc * 1e-3) / 1e9},
       "b64_decode": {"ms": t_dec, "GBps": (n + 4 * n // 3) / (t_dec * 1e-3) / 1e9},
       "words": W,
       "b64_words": {"ms": t_w, "GBps": 40 * W / (t_w * 1e-3) / 1e9},
       "b64_unwords": {"ms": t_uw, "GBps": 40 * W / (t_uw * 1e-3) / 1e9}}

# Beaver open exchange (MultiplicationExchangeObject.interimValues): 2W pairs
# of signed diffs <-> FactorPair JSON text, W = one 4 Mi-word C5 batch.
# Bytes counted: 34 B of diffs per pair + the text.
P2 = 2 * (1 << 22)
mag = ctx.synth_words(2, 2 * P2).view(P2, 2, 16)
neg = torch.randint(0, 2, (P2, 2), dtype=torch.uint8, device="cuda")
t_xe, (txt, ln) = timed(lambda: ctx.exchange_encode(mag, neg), reps=10)
nchars = int(ln.item())
arr = txt[:nchars]
t_xd, res = timed(lambda: ctx.exchange_decode(arr, P2), reps=10)
assert int(res[2].item()) == A._lib.AMPH_NO_FAILURE
assert torch.equal(res[0], mag)
# CPU reference point: Python's json module on a 100k-pair sample (1 thread)
import time  # noqa: E402
import numpy as np  # noqa: E402
sample = 100_000
m_h, n_h = mag[:sample].cpu().numpy(), neg[:sample].cpu().numpy()
vals = [int.from_bytes(m_h[k, j].tobytes(), "little") * (-1 if n_h[k, j] else 1)
        for k in range(sample) for j in range(2)]
t0 = time.perf_counter()
s = json.dumps([{"a": vals[2 * k], "b": vals[2 * k + 1]} for k in range(sample)], separators=(",", ":"))
t1 = time.perf_counter()
back = json.loads(s)
t2 = time.perf_counter()
out["exchange_pairs"] = P2
out["exchange_chars"] = nchars
out["exchange_encode"] = {"ms": t_xe, "GBps": (34 * P2 + nchars) / (t_xe * 1e-3) / 1e9,
                          "Mpairs_per_s": P2 / (t_xe * 1e-3) / 1e6}
out["exchange_decode"] = {"ms": t_xd, "GBps": (34 * P2 + nchars) / (t_xd * 1e-3) / 1e9,
                          "Mpairs_per_s": P2 / (t_xd * 1e-3) / 1e6}
out["exchange_cpu_python_json"] = {"pairs": sample, "encode_Mpairs_per_s": sample / (t1 - t0) / 1e6,
                                   "decode_Mpairs_per_s": sample / (t2 - t1) / 1e6}
# CPU reference point for base64: CPython's binascii (C, one thread; Jackson's
# MIME_NO_LINEFEEDS variant is the same alphabet and padding) on 96 MiB
import base64  # noqa: E402
b_h = raw[: 3 << 25].cpu().numpy().tobytes()
t0 = time.perf_counter()
e_h = base64.b64encode(b_h)
t1 = time.perf_counter()
base64.b64decode(e_h, validate=True)
t2 = time.perf_counter()
nb = len(b_h) + len(e_h)
out["b64_cpu_python_binascii"] = {"bytes": len(b_h), "encode_GBps": nb / (t1 - t0) / 1e9,
                                  "decode_GBps": nb / (t2 - t1) / 1e9, "threads": 1}
print(json.dumps(out))
