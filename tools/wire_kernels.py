"""Drive the fused wire kernels alone, for rocprofv3 kernel-trace / PMC passes
(VERDICT r3 item 5): k_mask_b64 (createSecret from the /input-masks text,
records out) and k_rv_b64 (getSecret from the share ODO text) on device
buffers, W words x N parties, REPS launches each after one warm-up.

    python tools/wire_kernels.py [--words 4194304] [--parties 3] [--reps 10]

Prints one JSON line: per-kernel average ms from HIP events on the launch
stream (amph_time_next_launch) and the algorithmic bytes per launch (text +
secrets + records / secrets out), so the profile's kernel durations and
FETCH_SIZE / WRITE_SIZE can be set against them."""
import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--words", type=int, default=4 << 20)
    ap.add_argument("--parties", type=int, default=3)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", choices=["mask", "rv", "both"], default="both")
    a = ap.parse_args()
    import torch
    import amphora_amd as A
    from amphora_amd.spdz import TEST_PRIME, TEST_R, TEST_RINV
    ctx = A.Context(TEST_PRIME, TEST_R, TEST_RINV, device=0)
    W, n = a.words, a.parties
    _, mbuf, _ = ctx.synth_odos(seed=1, n=n, words=W)
    _, sbuf, splain = ctx.synth_odos(seed=2, n=n, words=W, with_plain=True)
    secrets = ctx.synth_words(seed=3, count=W)
    mtext = [[ctx.base64_encode(mbuf[k, j].reshape(-1)) for k in range(5)] for j in range(n)]
    stext = [[ctx.base64_encode(sbuf[k, j].reshape(-1)) for k in range(5)] for j in range(n)]
    del mbuf, sbuf
    torch.cuda.synchronize()
    nchars = mtext[0][0].numel()
    text_bytes = 5 * n * nchars
    lib = A._lib
    res = {"words": W, "parties": n, "reps": a.reps, "nchars_per_field": nchars}

    def timed(fn):
        fn()  # warm-up
        torch.cuda.synchronize()
        evs = [(lib.TimingEvent(), lib.TimingEvent()) for _ in range(a.reps)]
        for e0, e1 in evs:
            lib.lib.amph_time_next_launch(e0.handle, e1.handle)
            fn()
        torch.cuda.synchronize()
        return sum(e0.elapsed_ms(e1) for e0, e1 in evs) / a.reps

    if a.only in ("mask", "both"):
        last = {}

        def mask():
            last["r"] = ctx.mask_input_b64(mtext, W, secrets, records=True, raw=False)
        ms = timed(mask)
        _, rec, ff, bad = last["r"]
        torch.cuda.synchronize()
        assert int(ff.item()) == lib.AMPH_NO_FAILURE and int(bad.item()) == lib.AMPH_NO_FAILURE
        b = text_bytes + 16 * W + 24 * W
        res["k_mask_b64"] = {"ms": round(ms, 5), "bytes": b, "GBps": round(b / ms / 1e6, 1),
                             "frac_8TBs": round(b / ms / 1e6 / 8000, 4)}
    if a.only in ("rv", "both"):
        last = {}

        def rv():
            last["r"] = ctx.recombine_verify_b64(stext, W)
        ms = timed(rv)
        y, ff, bad = last["r"]
        torch.cuda.synchronize()
        assert int(ff.item()) == lib.AMPH_NO_FAILURE and int(bad.item()) == lib.AMPH_NO_FAILURE
        assert torch.equal(y, splain), "k_rv_b64 secrets"
        b = text_bytes + 16 * W
        res["k_rv_b64"] = {"ms": round(ms, 5), "bytes": b, "GBps": round(b / ms / 1e6, 1),
                           "frac_8TBs": round(b / ms / 1e6 / 8000, 4)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
