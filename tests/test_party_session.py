"""One party's Output Delivery with device-resident state (amph_party_*,
include/amphora.h) against the C oracle, for every party of an N-party
exchange: y/r/v and the interimValues text after begin, w/u (or all five
fields as base64) after the partners' texts.  The texts are checked against
the oracle's diffs formatted as Jackson writes them (FactorPair list,
OutputDeliveryService.java:186-200), the results against recombineDiffs +
multiplySharedSecrets (:231-286) on the oracle.  Then the session's error
contract: missing / repeated / out-of-range partner slots, malformed and
short partner texts (the session stays usable), a second finish.
"""
import base64

import numpy as np
import pytest

from oracle import amphora_oracle as O

P, R, RINV = O.TEST_PRIME, O.TEST_R, O.TEST_RINV

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import amphora_amd as A
    return A.Context(P, R, RINV)


@pytest.fixture(scope="module")
def F():
    from oracle import coracle
    return coracle.test_field(threads=8)


def jackson_text(mag, neg) -> bytes:
    """The FactorPair JSON array of diffs (mag (P, 2, 16) LE, neg (P, 2))."""
    vals = []
    for k in range(mag.shape[0]):
        pair = []
        for j in range(2):
            x = int.from_bytes(mag[k, j].tobytes(), "little")
            pair.append(-x if neg[k, j] and x else x)
        vals.append('{"a":%d,"b":%d}' % tuple(pair))
    return ("[" + ",".join(vals) + "]").encode()


def party_inputs(F, n, W, stride=32):
    shares = [F.synth_words(seed=100 + j, count=W * stride // 16).reshape(W, stride) for j in range(n)]
    masks = [F.synth_words(seed=200 + j, count=4 * W).reshape(2 * W, 32) for j in range(n)]
    triples = [F.synth_words(seed=300 + j, count=12 * W).reshape(2 * W, 96) for j in range(n)]
    return shares, masks, triples


@pytest.mark.parametrize("n,W,stride", [(2, 777, 32), (3, 5000, 32), (3, 70001, 16), (1, 300, 32),
                                         (5, 3001, 32), (16, 513, 16)])
def test_session_matches_oracle(ctx, F, n, W, stride):
    shares, masks, triples = party_inputs(F, n, W, stride)
    pre = [F.odo_pre(shares[j], stride, masks[j], triples[j]) for j in range(n)]
    sessions, texts = [], []
    for j in range(n):
        s = ctx.party_begin(shares[j], stride, masks[j], triples[j], n)
        oy, orr, ov, omag, oneg = pre[j]
        assert np.array_equal(s.y, oy) and np.array_equal(s.r, orr) and np.array_equal(s.v, ov)
        t = s.text()
        if W <= 5000:
            assert t == jackson_text(omag, oneg)
        assert t == ctx.exchange_encode(omag, oneg)  # the host-path encoder (Jackson-pinned in test_wire)
        sessions.append(s)
        texts.append(t)
    for j, s in enumerate(sessions):
        others = [k for k in range(n) if k != j]
        for slot, k in enumerate(reversed(others), start=1):  # partner order is free: the sum commutes
            s.partner(slot, texts[k])
        order = [j] + others
        opened = F.recombine_diffs([pre[k][3] for k in order], [pre[k][4] for k in order])
        ow, ou = F.odo_post(opened, triples[j], j == 0)
        if j == n - 1:  # the last party takes the whole response as base64 text
            got = s.finish_b64(j == 0)
            want = [base64.b64encode(x.tobytes()) for x in (pre[j][0], pre[j][1], pre[j][2], ow, ou)]
            assert got == want
        else:
            w, u = s.finish(j == 0)
            assert np.array_equal(w, ow) and np.array_equal(u, ou)
        s.close()


def test_session_errors(ctx, F):
    import amphora_amd as A
    n, W = 3, 1000
    shares, masks, triples = party_inputs(F, n, W)
    s0 = ctx.party_begin(shares[0], 32, masks[0], triples[0], n, want_yrv=False)
    s1 = ctx.party_begin(shares[1], 32, masks[1], triples[1], n)
    s2 = ctx.party_begin(shares[2], 32, masks[2], triples[2], n)
    assert s0.y is None
    t1, t2 = s1.text(), s2.text()
    with pytest.raises(A.AmphoraNativeError, match="partner slot 1's interimValues text is missing"):
        s0.finish(True)
    for slot in (0, 3, -1):
        with pytest.raises(A.AmphoraNativeError, match=r"partner slot must be in \[1, 2\]"):
            s0.partner(slot, t1)
    # malformed: a digit replaced -> rejected at its offset, the slot stays free
    at = t1.index(b":") + 3
    bad = t1[:at] + b"x" + t1[at + 1:]
    with pytest.raises(ValueError, match="Malformed FactorPair JSON at offset") as ei:
        s0.partner(1, bad)
    assert 6 <= int(str(ei.value).rsplit(" ", 1)[1]) <= at  # the token holding the bad byte
    # one pair short -> a count error
    short = t1[: t1.rindex(b",{")] + b"]"
    with pytest.raises(ValueError, match="exactly %d FactorPairs" % (2 * W)):
        s0.partner(1, short)
    s0.partner(1, t1)
    with pytest.raises(A.AmphoraNativeError, match="slot 1 already holds a text"):
        s0.partner(1, t2)
    with pytest.raises(A.AmphoraNativeError, match="partner slot 2's interimValues text is missing"):
        s0.finish(True)
    s0.partner(2, t2)
    w, u = s0.finish(True)
    pre = [F.odo_pre(shares[j], 32, masks[j], triples[j]) for j in range(n)]
    opened = F.recombine_diffs([p[3] for p in pre], [p[4] for p in pre])
    ow, ou = F.odo_post(opened, triples[0], True)
    assert np.array_equal(w, ow) and np.array_equal(u, ou)
    with pytest.raises(A.AmphoraNativeError, match="already finished"):
        s0.finish(True)
    for s in (s0, s1, s2):
        s.close()
    # argument checks before any device work
    with pytest.raises(A.AmphoraNativeError, match=r"n_parties must be in \[1, 16\]"):
        ctx.party_begin(shares[0], 32, masks[0], triples[0], 17)
    with pytest.raises(A.AmphoraNativeError, match="expected 2000 multiplication triples"):
        ctx.party_begin(shares[0], 32, masks[0], triples[0][:10], 2)


def test_session_empty(ctx):
    """words = 0: the text is "[]", an empty partner text completes the exchange."""
    z = np.zeros((0, 32), np.uint8)
    s = ctx.party_begin(z, 32, np.zeros((0, 32), np.uint8), np.zeros((0, 96), np.uint8), 2)
    assert s.text() == b"[]"
    s.partner(1, b"[]")
    w, u = s.finish(False)
    assert w.shape == (0, 16) and u.shape == (0, 16)
    s.close()


def reorder_text(t: bytes) -> bytes:
    """The same FactorPairs with "b" listed before "a" (a JSON reader accepts
    either member order; the span-form decode keeps text order and k_open_post
    swaps the pair back by its key bit)."""
    import re
    return re.sub(rb'\{"a":(-?\d+),"b":(-?\d+)\}', rb'{"b":\2,"a":\1}', t)


def test_session_partner_text_forms(ctx, F):
    """Every partner text form decodes to the same diffs: Jackson's compact
    text (span form), members swapped (span form, swapped back by finish),
    whitespace between tokens (the general pass: pair order), and a mix of
    partners in both forms in one finish."""
    n, W = 3, 20000
    shares, masks, triples = party_inputs(F, n, W)
    pre = [F.odo_pre(shares[j], 32, masks[j], triples[j]) for j in range(n)]
    texts = [ctx.party_begin(shares[j], 32, masks[j], triples[j], n).text() for j in range(1, n)]
    opened = F.recombine_diffs([p[3] for p in pre], [p[4] for p in pre])
    ow, ou = F.odo_post(opened, triples[0], True)
    forms = {
        "compact": texts,
        "swapped": [reorder_text(t) for t in texts],
        "spaced": [t.replace(b',"b"', b', "b"').replace(b"},{", b"},\n{") for t in texts],
        "mixed": [reorder_text(texts[0]), texts[1].replace(b":", b": ")],
    }
    for name, ts in forms.items():
        s = ctx.party_begin(shares[0], 32, masks[0], triples[0], n, want_yrv=False)
        for slot, t in enumerate(ts, start=1):
            s.partner(slot, t)
        w, u = s.finish(True)
        assert np.array_equal(w, ow) and np.array_equal(u, ou), name
        s.close()


def test_session_partner_text_forms_many_parties(ctx, F):
    """Party counts past k_open_post's templated 1-4: six parties (five
    partners) and sixteen (AMPH_MAX_PARTIES, fifteen partners), the partner
    texts cycling through the compact (span form), member-swapped (span form)
    and spaced (pair order) forms, so one finish sums span-form and
    pair-order partners at a run-time party count."""
    for n, W in ((6, 6007), (16, 1031)):
        shares, masks, triples = party_inputs(F, n, W)
        pre = [F.odo_pre(shares[j], 32, masks[j], triples[j]) for j in range(n)]
        texts = [ctx.exchange_encode(pre[j][3], pre[j][4]) for j in range(1, n)]
        forms = [lambda t: t, reorder_text, lambda t: t.replace(b"},{", b"}, {")]
        opened = F.recombine_diffs([p[3] for p in pre], [p[4] for p in pre])
        for p0 in (True, False):
            ow, ou = F.odo_post(opened, triples[0], p0)
            s = ctx.party_begin(shares[0], 32, masks[0], triples[0], n, want_yrv=False)
            for slot, t in enumerate(texts, start=1):
                s.partner(slot, forms[(slot + p0) % 3](t))
            w, u = s.finish(p0)
            assert np.array_equal(w, ow) and np.array_equal(u, ou), (n, p0)
            s.close()


def test_session_small_diffs(ctx, F):
    """Triples whose a, b equal the words they are subtracted from: every diff
    is 0, the texts are {"a":0,"b":0} runs (over 1000 values per 8 KiB, more
    than a span's slots: the general pass decodes them), and the products are
    the c shares (+ nothing): checked against the oracle."""
    n, W = 2, 9000
    shares, masks, triples = party_inputs(F, n, W)
    for j in range(n):
        t = triples[j].copy()
        t[0::2, 0:16] = shares[j][:, 0:16]
        t[0::2, 32:48] = masks[j][0::2, 0:16]
        t[1::2, 0:16] = masks[j][1::2, 0:16]
        t[1::2, 32:48] = masks[j][0::2, 0:16]
        triples[j] = t
    pre = [F.odo_pre(shares[j], 32, masks[j], triples[j]) for j in range(n)]
    assert not pre[0][3].any()
    s0 = ctx.party_begin(shares[0], 32, masks[0], triples[0], n)
    s1 = ctx.party_begin(shares[1], 32, masks[1], triples[1], n)
    t1 = s1.text()
    assert t1.startswith(b'[{"a":0,"b":0},{"a":0,"b":0}')
    s0.partner(1, t1)
    w, u = s0.finish(True)
    opened = F.recombine_diffs([p[3] for p in pre], [p[4] for p in pre])
    ow, ou = F.odo_post(opened, triples[0], True)
    assert np.array_equal(w, ow) and np.array_equal(u, ou)
    s0.close()
    s1.close()


@pytest.mark.parametrize("n,W,stride", [(3, 5000, 32), (2, 70001, 16), (6, 4099, 32), (16, 257, 16)])
def test_session_device_mode(ctx, F, n, W, stride):
    """amph_party_*_dev on torch device tensors, texts handed between the
    parties on the device: the five base64 fields equal the host session's /
    the oracle's."""
    import torch
    shares, masks, triples = party_inputs(F, n, W, stride)
    pre = [F.odo_pre(shares[j], stride, masks[j], triples[j]) for j in range(n)]
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    inputs = [(dev(shares[j]), dev(masks[j]), dev(triples[j])) for j in range(n)]
    sessions = [ctx.party_begin_dev(*inputs[j][:1], stride, *inputs[j][1:], n) for j in range(n)]
    texts = []
    for j, s in enumerate(sessions):
        t, ln = s.text_dev()
        texts.append((t, ln))
        if j == 0 and W <= 5000:
            assert s.text() == jackson_text(pre[0][3], pre[0][4])
    lens = [int(ln.item()) for _, ln in texts]
    for j, s in enumerate(sessions):
        others = [k for k in range(n) if k != j]
        bads = [s.partner(slot, texts[k][0][:lens[k]]) for slot, k in enumerate(others, start=1)]
        fields = s.finish_b64(j == 0)
        torch.cuda.synchronize()
        assert all(int(b.item()) == 0x7F7F7F7F7F7F7F7F for b in bads)
        opened = F.recombine_diffs([pre[k][3] for k in [j] + others], [pre[k][4] for k in [j] + others])
        ow, ou = F.odo_post(opened, triples[j], j == 0)
        want = [base64.b64encode(x.tobytes()) for x in (pre[j][0], pre[j][1], pre[j][2], ow, ou)]
        assert [f.cpu().numpy().tobytes() for f in fields] == want
    for s in sessions:
        s.close()


def test_session_device_mode_errors(ctx, F):
    """A malformed partner text is reported in the device word; host calls on a
    device-mode session (and the reverse) are refused."""
    import torch
    import amphora_amd as A
    n, W = 2, 3000
    shares, masks, triples = party_inputs(F, n, W)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    s = ctx.party_begin_dev(dev(shares[0]), 32, dev(masks[0]), dev(triples[0]), n)
    t1 = ctx.party_begin(shares[1], 32, masks[1], triples[1], n).text()
    at = t1.index(b":") + 3
    bad_text = t1[:at] + b"x" + t1[at + 1:]
    bad = s.partner(1, dev(np.frombuffer(bad_text, np.uint8).copy()))
    assert 6 <= int(bad.item()) <= at
    with pytest.raises(A.AmphoraNativeError, match="takes the \\*_dev calls"):
        A._lib.PartySession.finish(s, True)
    h = ctx.party_begin(shares[1], 32, masks[1], triples[1], n)
    import ctypes as C
    t, ln = C.c_void_p(), C.c_void_p()
    assert A._lib.lib.amph_party_text_dev(h._h, C.byref(t), C.byref(ln)) == A._lib.AMPH_E_PARAM
    assert b"host-mode party session takes the host calls" in A._lib.lib.amph_last_error()
    s.close()
    h.close()


def test_text_length_edges(ctx, F):
    """A partner text whose length ends a few bytes short of an 8 KiB span
    boundary (trailing whitespace pads it: len % 8192 = 8180), decoded in host
    mode, in device mode at an odd device address (the span count then covers
    one span past the text), and by the pair-order decode (amph_exchange_decode,
    host and device): the same diffs / w, u as the compact text."""
    import torch
    n, W = 2, 3000
    shares, masks, triples = party_inputs(F, n, W)
    pre = [F.odo_pre(shares[j], 32, masks[j], triples[j]) for j in range(n)]
    t1 = ctx.party_begin(shares[1], 32, masks[1], triples[1], n).text()
    tp = t1 + b" " * ((8180 - len(t1) % 8192) % 8192)
    assert len(tp) % 8192 == 8180
    opened = F.recombine_diffs([p[3] for p in pre], [p[4] for p in pre])
    ow, ou = F.odo_post(opened, triples[0], True)
    for text in (t1, tp):
        s = ctx.party_begin(shares[0], 32, masks[0], triples[0], n, want_yrv=False)
        s.partner(1, text)
        w, u = s.finish(True)
        assert np.array_equal(w, ow) and np.array_equal(u, ou)
        s.close()
        m, g = ctx.exchange_decode(text, 2 * W)
        assert ctx.exchange_encode(m, g) == t1
        for off in (0, 5):
            buf = torch.zeros(len(text) + off, dtype=torch.uint8, device="cuda")
            buf[off:] = torch.from_numpy(np.frombuffer(text, np.uint8).copy()).cuda()
            dm, dg, bad = ctx.exchange_decode(buf[off:], 2 * W)
            torch.cuda.synchronize()
            assert int(bad.item()) == 0x7F7F7F7F7F7F7F7F
            assert ctx.exchange_encode(dm.cpu().numpy(), dg.cpu().numpy()) == t1
            dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
            sd = ctx.party_begin_dev(dev(shares[0]), 32, dev(masks[0]), dev(triples[0]), n)
            b = sd.partner(1, buf[off:])
            fields = sd.finish_b64(True)
            torch.cuda.synchronize()
            assert int(b.item()) == 0x7F7F7F7F7F7F7F7F
            assert fields[3].cpu().numpy().tobytes() == base64.b64encode(ow.tobytes())
            assert fields[4].cpu().numpy().tobytes() == base64.b64encode(ou.tobytes())
            sd.close()


def test_session_partner_fuzz_matches_pair_decode(ctx, F):
    """Mutated partner texts (a byte replaced, deleted or inserted, whitespace
    added): the session's one-read span-form decode accepts exactly the texts
    the pair-order decode (amph_exchange_decode: count pass + compact pass +
    general pass) accepts, reports the same error at the same offset, and on
    an accepted text finishes with the w, u the oracle computes from that
    decode's diffs."""
    rng = np.random.default_rng(7)
    n, W = 2, 1500
    shares, masks, triples = party_inputs(F, n, W)
    pre0 = F.odo_pre(shares[0], 32, masks[0], triples[0])
    t1 = ctx.party_begin(shares[1], 32, masks[1], triples[1], n).text()
    alphabet = list(b'0123456789-,:{}[]"ab \n')
    accepted = rejected = 0
    for trial in range(80):
        t = bytearray(t1)
        pos = int(rng.integers(0, len(t)))
        kind = trial % 4
        if kind == 0:
            t[pos] = int(rng.choice(alphabet))
        elif kind == 1:
            del t[pos]
        elif kind == 2:
            t.insert(pos, int(rng.choice(list(b' 0-,'))))
        else:
            t[pos:pos] = b" \t"
        t = bytes(t)
        try:
            m, g = ctx.exchange_decode(t, 2 * W)
            ref = None
        except ValueError as e:
            ref = str(e)
        s = ctx.party_begin(shares[0], 32, masks[0], triples[0], n, want_yrv=False)
        try:
            s.partner(1, t)
            got = None
        except ValueError as e:
            got = str(e)
        assert got == ref, (trial, kind, pos)
        if ref is None:
            accepted += 1
            w, u = s.finish(True)
            opened = F.recombine_diffs([pre0[3], m], [pre0[4], g])
            ow, ou = F.odo_post(opened, triples[0], True)
            assert np.array_equal(w, ow) and np.array_equal(u, ou), (trial, kind, pos)
        else:
            rejected += 1
        s.close()
    assert accepted > 5 and rejected > 5


def test_session_device_mode_rejected_text_poisons_and_resubmits(ctx, F):
    """A device-mode partner text whose verdict word reports a failure: a
    finish that runs anyway writes poisoned fields ("!!!!" first, no base64
    decoder accepts them); after amph_party_reset_partner the slot takes a
    good text and the fields equal the oracle's (the slot was
    marked filled before the verdict was known)."""
    import torch
    n, W = 2, 3000
    shares, masks, triples = party_inputs(F, n, W)
    pre = [F.odo_pre(shares[j], 32, masks[j], triples[j]) for j in range(n)]
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    t1 = ctx.party_begin(shares[1], 32, masks[1], triples[1], n).text()
    at = t1.index(b":") + 3
    bad_text = dev(np.frombuffer(t1[:at] + b"x" + t1[at + 1:], np.uint8).copy())
    good_text = dev(np.frombuffer(t1, np.uint8).copy())
    # finish after a rejected text: poisoned output
    s = ctx.party_begin_dev(dev(shares[0]), 32, dev(masks[0]), dev(triples[0]), n)
    bad = s.partner(1, bad_text)
    fields = s.finish_b64(True)
    torch.cuda.synchronize()
    assert int(bad.item()) != 0x7F7F7F7F7F7F7F7F
    for f in fields:
        assert f[:4].cpu().numpy().tobytes() == b"!!!!"
    s.close()
    # reject, reset the slot, resubmit: exact output
    s = ctx.party_begin_dev(dev(shares[0]), 32, dev(masks[0]), dev(triples[0]), n)
    bad = s.partner(1, bad_text)
    torch.cuda.synchronize()
    assert int(bad.item()) != 0x7F7F7F7F7F7F7F7F
    s.reset_partner(1)
    bad = s.partner(1, good_text)
    fields = s.finish_b64(True)
    torch.cuda.synchronize()
    assert int(bad.item()) == 0x7F7F7F7F7F7F7F7F
    opened = F.recombine_diffs([pre[0][3], pre[1][3]], [pre[0][4], pre[1][4]])
    ow, ou = F.odo_post(opened, triples[0], True)
    want = [base64.b64encode(x.tobytes()) for x in (pre[0][0], pre[0][1], pre[0][2], ow, ou)]
    assert [f.cpu().numpy().tobytes() for f in fields] == want
    s.close()


def test_session_pool_reclaimed_on_out_of_memory(F):
    """the party-session buffers the context pools after
    amph_party_free must not cause an out-of-memory error.  Sessions of
    growing sizes fill the pool; the GPU is then filled so that the next,
    larger session fits only if the pooled buffers are freed first -- it
    must begin, with the pool emptied.  Also: the pool never exceeds
    AMPH_PARTY_POOL_BYTES (here the 32 GiB default is not reached)."""
    import torch
    import amphora_amd as A
    c = A.Context(P, R, RINV)
    n = 2

    def dev_inputs(W, seed):
        sh = c.synth_words(seed=seed, count=2 * W).view(W, 32)
        mk = c.synth_words(seed=seed + 1, count=4 * W).view(2 * W, 32)
        tr = c.synth_words(seed=seed + 2, count=12 * W).view(2 * W, 96)
        return sh, mk, tr

    sizes = [1 << 18, 1 << 19, 1 << 20]
    for i, W in enumerate(sizes):
        sh, mk, tr = dev_inputs(W, 10 * i)
        s = c.party_begin_dev(sh, 32, mk, tr, n)
        torch.cuda.synchronize()
        s.close()
        del sh, mk, tr
    st = c.stats()
    assert st["pool_buffers"] >= len(sizes) and st["pool_bytes"] > 0
    pooled = st["pool_bytes"]
    big = 1 << 21
    sh, mk, tr = dev_inputs(big, 99)
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    # the big session's buffer ~ 2x the 1 Mi-word session's, the largest pooled
    need = 2 * max_pooled_estimate(pooled, sizes)
    free, _ = torch.cuda.mem_get_info()
    leave = need - pooled // 3  # < need, but need <= leave + pooled
    filler = torch.empty(max(0, free - leave), dtype=torch.uint8, device="cuda")
    try:
        s = c.party_begin_dev(sh, 32, mk, tr, n)
        torch.cuda.synchronize()
        st2 = c.stats()
        s.close()
    finally:
        del filler
        torch.cuda.empty_cache()
    assert st2["pool_buffers"] == 0, st2


def max_pooled_estimate(pooled, sizes):
    """Bytes of the largest pooled session buffer: sizes double, so it is
    W_max / sum(W) of the pooled bytes."""
    return pooled * sizes[-1] // sum(sizes)


def test_session_device_mode_keeps_its_own_verdicts(ctx, F):
    """the partner verdict finish_b64_dev checks is the session's
    own copy, taken on the partner call's stream, and finish waits for that
    call's work even on another stream.  So after the partner call the caller
    may overwrite its bad_index word: a rejected text still poisons the
    fields, an accepted one is not poisoned by a later write into the word."""
    import torch
    n, W = 2, 3000
    shares, masks, triples = party_inputs(F, n, W)
    pre = [F.odo_pre(shares[j], 32, masks[j], triples[j]) for j in range(n)]
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    t1 = ctx.party_begin(shares[1], 32, masks[1], triples[1], n).text()
    at = t1.index(b":") + 3
    bad_text = dev(np.frombuffer(t1[:at] + b"x" + t1[at + 1:], np.uint8).copy())
    good_text = dev(np.frombuffer(t1, np.uint8).copy())
    opened = F.recombine_diffs([pre[0][3], pre[1][3]], [pre[0][4], pre[1][4]])
    ow, ou = F.odo_post(opened, triples[0], True)
    want = [base64.b64encode(x.tobytes()) for x in (pre[0][0], pre[0][1], pre[0][2], ow, ou)]
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    for text, poisoned in ((bad_text, True), (good_text, False)):
        torch.cuda.synchronize()
        s = ctx.party_begin_dev(dev(shares[0]), 32, dev(masks[0]), dev(triples[0]), n)
        torch.cuda.synchronize()
        word = torch.empty(1, dtype=torch.int64, device="cuda")
        with torch.cuda.stream(sa):
            s.partner(1, text, bad=word)
            # the caller reuses its word right after the call (same stream)
            word.fill_(0x7F7F7F7F7F7F7F7F if poisoned else 5)
        with torch.cuda.stream(sb):
            fields = s.finish_b64(True)
        torch.cuda.synchronize()
        got = [f.cpu().numpy().tobytes() for f in fields]
        if poisoned:
            assert all(g[:4] == b"!!!!" for g in got)
        else:
            assert got == want
        s.close()
