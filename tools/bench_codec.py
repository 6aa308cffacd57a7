"""Device-resident throughput of the base64 wire codec kernels (tool).
Bytes counted: input read + output written (algorithmic)."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import amphora_amd as A  # noqa: E402
from oracle.amphora_oracle import TEST_PRIME, TEST_R, TEST_RINV  # noqa: E402

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
print(json.dumps(out))
