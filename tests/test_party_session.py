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


@pytest.mark.parametrize("n,W,stride", [(2, 777, 32), (3, 5000, 32), (3, 70001, 16), (1, 300, 32)])
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
