"""K_RV / K_MASK straight from the base64 wire text (amph_recombine_verify_b64,
amph_mask_input_b64) against the C oracle on the decoded words and Python's
base64 module (Jackson's MIME_NO_LINEFEEDS variant: standard alphabet, '='
padding, no line breaks):

* getSecret: VerifiableSecretShare fields (VerifiableSecretTest.java:41-90)
  -> verifyOutputDeliveryObjects (DefaultAmphoraClient.java:206-217, 476-505);
* createSecret: OutputDeliveryObject fields -> verify + maskInput -> the
  {"value": base64} records of MaskedInputData (:150-170, MaskedInputData.java:44-52).

Word counts straddle the 768-word workgroups and the three padding cases
(16 W mod 3 = 0, 1, 2); party counts cover the templated (1-4) and run-time
paths; bad characters are placed in every field, in the padding group and
past the fast-path workgroups.
"""
import base64

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from oracle import amphora_oracle as O  # noqa: E402
from oracle import coracle  # noqa: E402

P, R, RINV = O.TEST_PRIME, O.TEST_R, O.TEST_RINV


@pytest.fixture(scope="module")
def ctx():
    import torch
    assert torch.cuda.is_available()
    import amphora_amd as A
    return A.Context(P, R, RINV)


@pytest.fixture(scope="module")
def F():
    return coracle.test_field(threads=8)


def texts_of(odos):
    return [[base64.b64encode(np.ascontiguousarray(f).tobytes()) for f in o] for o in odos]


def on_device(texts):
    import torch
    return [[torch.frombuffer(bytearray(t), dtype=torch.uint8).cuda() for t in o] for o in texts]


def _rv(ctx, texts, W, mode):
    if mode == "host":
        return ctx.recombine_verify_b64(texts, W)
    y, ff, bad = ctx.recombine_verify_b64(on_device(texts), W)
    import torch
    torch.cuda.synchronize()
    nf = 0x7F7F7F7F7F7F7F7F
    ffv, badv = int(ff.item()), int(bad.item())
    return y.cpu().numpy(), (-1 if ffv == nf else ffv), (-1 if badv == nf else badv)


@pytest.mark.parametrize("mode", ["host", "device"])
@pytest.mark.parametrize("n,W", [(2, 1), (2, 2), (2, 3), (1, 767), (2, 768), (3, 769), (4, 1537),
                                 (2, 2304), (5, 2000), (2, 100_003), (3, 65_536), (16, 1031)])
def test_rv_b64_matches_oracle(ctx, F, mode, n, W):
    odos, _ = F.synth_odos(seed=700 + n + W, n=n, W=W, noncanon_permille=20)
    y, ff, bad = _rv(ctx, texts_of(odos), W, mode)
    oy, off = F.recombine_verify(odos)
    assert ff == off == -1 and bad == -1 and np.array_equal(y, oy)
    fault = (W * 2) // 3
    odos, _ = F.synth_odos(seed=800 + n + W, n=n, W=W, fault_index=fault)
    y, ff, bad = _rv(ctx, texts_of(odos), W, mode)
    assert ff == fault and bad == -1


@pytest.mark.parametrize("mode", ["host", "device"])
@pytest.mark.parametrize("W", [4000, 4001, 4002])  # padding 0 / 2 / 1 ('' / '==' / '=')
@pytest.mark.parametrize("n", [3, 5])  # 5: the runtime party-count kernels (NP = 0), same LDS-table decode
def test_rv_b64_bad_characters(ctx, F, mode, W, n):
    odos, _ = F.synth_odos(seed=900 + W + n, n=n, W=W)
    base = texts_of(odos)
    nchars = len(base[0][0])
    assert nchars == 4 * ((16 * W + 2) // 3)
    pad = (3 - (16 * W) % 3) % 3
    cases = [(0, 0, 0, b"*"), (1, 3, 5000, b"-"), (2, 4, nchars - 1 - pad, b"="),
             (1, 2, nchars // 2, b"\x80"), (0, 1, 16 * 1024 * 3 + 7, b" ")]
    if pad:
        cases.append((2, 0, nchars - 1, b"A"))  # a character where '=' must be
    else:
        cases.append((2, 0, nchars - 1, b"="))  # '=' where no padding is due
    for j, k, pos, ch in cases:
        texts = [list(o) for o in base]
        t = bytearray(texts[j][k])
        t[pos] = ch[0]
        texts[j][k] = bytes(t)
        exp = (5 * j + k) * nchars + pos
        if mode == "host":
            with pytest.raises(ValueError, match="index %d of party %d's" % (pos, j)):
                ctx.recombine_verify_b64(texts, W)
        else:
            _, _, bad = _rv(ctx, texts, W, mode)
            assert bad == exp, (j, k, pos, ch)
    # two bad characters: the smaller (field, offset) wins
    texts = [list(o) for o in base]
    for j, k, pos in ((2, 1, 10), (1, 4, 20)):
        t = bytearray(texts[j][k])
        t[pos] = ord("!")
        texts[j][k] = bytes(t)
    _, _, bad = _rv(ctx, texts, W, "device")
    assert bad == (5 * 1 + 4) * nchars + 20


_B64 = frozenset(b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/")


def _first_bad(t: bytes, pad: int) -> int:
    """Offset of the first character Jackson's MIME_NO_LINEFEEDS decoder
    rejects: outside the alphabet before the padding, anything but '=' in
    it; -1 if none."""
    body = len(t) - pad
    for i, c in enumerate(t):
        if (c not in _B64) if i < body else (c != ord("=")):
            return i
    return -1


@pytest.mark.parametrize("W", [64, 65, 66])  # padding '==' / '=' / ''
@pytest.mark.parametrize("n", [2, 5])
def test_rv_b64_mutations(ctx, F, W, n):
    """Random single-character replacements in a random party's random field:
    an invalid character is reported at its (5 party + field) nchars +
    offset; a valid one changes the decoded word (Python's base64 says how),
    and the verdict and secrets equal the C oracle's on those words."""
    import random
    rng = random.Random(W + n)
    odos, _ = F.synth_odos(seed=1200 + W + n, n=n, W=W)
    base = texts_of(odos)
    nchars = len(base[0][0])
    pad = (3 - (16 * W) % 3) % 3
    alphabet = sorted(_B64)
    for _ in range(150):
        j, k, pos = rng.randrange(n), rng.randrange(5), rng.randrange(nchars)
        r = rng.random()
        ch = alphabet[rng.randrange(64)] if r < 0.5 else ord("=") if r < 0.7 else rng.randrange(256)
        t = bytearray(base[j][k])
        t[pos] = ch
        texts = [list(o) for o in base]
        texts[j][k] = bytes(t)
        y, ff, bad = _rv(ctx, texts, W, "device")
        fb = _first_bad(bytes(t), pad)
        if fb >= 0:
            assert bad == (5 * j + k) * nchars + fb, (j, k, pos, ch)
            continue
        assert bad == -1, (j, k, pos, ch)
        words = [list(o) for o in odos]
        words[j][k] = np.frombuffer(base64.b64decode(bytes(t), validate=True), np.uint8).reshape(W, 16)
        oy, off = F.recombine_verify([tuple(o) for o in words])
        assert ff == off, (j, k, pos, ch)
        if off < 0:
            assert np.array_equal(y, oy)


def test_rv_b64_length_checks(ctx, F):
    import amphora_amd as A
    odos, _ = F.synth_odos(seed=950, n=2, W=100)
    texts = texts_of(odos)
    with pytest.raises(A.AmphoraNativeError, match="expected"):
        ctx.recombine_verify_b64(texts, 101)
    short = [list(o) for o in texts]
    short[1][2] = short[1][2][:-4]
    with pytest.raises(A.AmphoraNativeError, match="same length"):
        ctx.recombine_verify_b64(short, 100)
    y, ff, bad = ctx.recombine_verify_b64([[b""] * 5, [b""] * 5], 0)
    assert y.shape == (0, 16) and ff == bad == -1


@pytest.mark.parametrize("mode", ["host", "device"])
@pytest.mark.parametrize("n,W,S", [(2, 1, 1), (2, 768, 768), (3, 1000, 999), (2, 100_003, 100_003),
                                   (4, 5000, 3000), (6, 800, 800), (2, 2305, 0), (16, 1031, 700)])
def test_mask_b64_matches_oracle(ctx, F, mode, n, W, S):
    import torch
    odos, _ = F.synth_odos(seed=1000 + n + W, n=n, W=W, noncanon_permille=10)
    secrets = F.synth_words(seed=1100 + W, count=S, mont=False)
    secrets[::7] = 0xFF  # any 128-bit value, reduced mod p
    exp = F.mask_input(secrets, [tuple(f[:S] for f in o) for o in odos])[0] if S else np.zeros((0, 16), np.uint8)
    texts = texts_of(odos)
    if mode == "host":
        m16, rec, ff, bad = ctx.mask_input_b64(texts, W, secrets, records=True, raw=True)
    else:
        m16, rec, ff, bad = ctx.mask_input_b64(on_device(texts), W, torch.from_numpy(secrets).cuda(),
                                               records=True, raw=True)
        torch.cuda.synchronize()
        m16, rec = m16.cpu().numpy(), rec.cpu().numpy()
        ff, bad = int(ff.item()), int(bad.item())
        ff = -1 if ff == 0x7F7F7F7F7F7F7F7F else ff
        bad = -1 if bad == 0x7F7F7F7F7F7F7F7F else bad
    assert ff == -1 and bad == -1
    assert np.array_equal(m16, exp)
    assert [r.tobytes() for r in rec[:500]] == [base64.b64encode(w.tobytes()) for w in exp[:500]]
    assert np.array_equal(rec, ctx.base64_encode_words(exp)) if S else rec.shape == (0, 24)
    # a fault past the secrets is still found (every mask word is verified)
    fault = W - 1
    odos, _ = F.synth_odos(seed=1200 + n + W, n=n, W=W, fault_index=fault)
    if mode == "host":
        _, _, ff, _ = ctx.mask_input_b64(texts_of(odos), W, secrets)
        assert ff == fault


@pytest.mark.parametrize("n,W", [(2, 1 << 20), (3, 1 << 24), (2, 1 << 26)])
def test_wire_kernels_at_baseline_sizes(ctx, n, W):
    """C2, C3 and the whole of C4 on one GPU: the parties' fields base64-coded
    on the GPU, then K_RV / K_MASK from the text must equal K_RV / K_MASK on
    the words (every output word), and an injected MAC fault is found at its
    index -- size-independent properties at the sizes BASELINE names."""
    import torch
    nf = 0x7F7F7F7F7F7F7F7F
    odos, buf, _ = ctx.synth_odos(seed=77, n=n, words=W, noncanon_permille=5)
    texts = [[ctx.base64_encode(f.reshape(-1)) for f in o] for o in odos]
    y_ref, ff_ref = ctx.recombine_verify(odos)
    y, ff, bad = ctx.recombine_verify_b64(texts, W)
    torch.cuda.synchronize()
    assert int(ff.item()) == int(ff_ref.item()) == nf and int(bad.item()) == nf
    assert torch.equal(y, y_ref)
    del y, y_ref
    secrets = ctx.synth_words(seed=78, count=W)
    m_ref, _ = ctx.mask_input(odos, secrets)
    m16, rec, ff, bad = ctx.mask_input_b64(texts, W, secrets, records=True, raw=True)
    torch.cuda.synchronize()
    assert int(ff.item()) == nf and int(bad.item()) == nf and torch.equal(m16, m_ref)
    assert torch.equal(rec, ctx.base64_encode_words(m_ref))
    del m16, rec, m_ref, secrets, texts
    # a MAC fault in party 1's w field, re-encoded
    fault = (2 * W) // 3
    odos[1][3][fault, 0] ^= 1
    texts = [[ctx.base64_encode(f.reshape(-1)) for f in o] for o in odos]
    _, ff, bad = ctx.recombine_verify_b64(texts, W)
    torch.cuda.synchronize()
    assert int(ff.item()) == fault and int(bad.item()) == nf
    del buf, odos, texts
    torch.cuda.empty_cache()


_ALPHABET = b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/"


def test_b64_every_character_in_every_unit_position(ctx, F):
    """The fused kernels' decode (b64.hpp dec4_values6: 6-bit value path, '/'
    routed through the roll selector) character by character, on the fast
    path (the first workgroup's units): every alphabet character at each of
    a unit's 16 positions must decode as Python's base64 says -- K_RV's
    secrets and verdict and K_MASK's masked words equal the oracle on the
    decoded words -- and each of the 192 other byte values, placed at a
    different unit position each, must be reported at exactly its offset."""
    import torch
    n, W = 2, 1536
    odos, _ = F.synth_odos(seed=1300, n=n, W=W)
    base = texts_of(odos)
    nchars = len(base[0][0])
    assert 16 * 64 < 16 * 256 <= nchars - 4096  # inside the first (fast) workgroup
    # unit u, position q holds alphabet[(u + 5 q) % 64]: every character at every position
    t = bytearray(base[1][0])  # party 1's y field: it reaches K_RV's and K_MASK's outputs
    for u in range(64):
        for q in range(16):
            t[16 * u + q] = _ALPHABET[(u + 5 * q) % 64]
    texts = [list(o) for o in base]
    texts[1][0] = bytes(t)
    words = [list(o) for o in odos]
    words[1][0] = np.frombuffer(base64.b64decode(bytes(t), validate=True), np.uint8).reshape(W, 16)
    y, ff, bad = _rv(ctx, texts, W, "device")
    oy, off = F.recombine_verify([tuple(o) for o in words])
    # (the replaced words break the MAC: both report the same first word; the
    # secrets of every word are written either way)
    assert bad == -1 and ff == off and np.array_equal(y, oy)
    secrets = F.synth_words(seed=1301, count=W, mont=False)
    m16, _, ffm, badm = ctx.mask_input_b64(on_device(texts), W, torch.from_numpy(secrets).cuda(), raw=True)
    torch.cuda.synchronize()
    exp, offm = F.mask_input(secrets, [tuple(o) for o in words])
    assert int(badm.item()) == 0x7F7F7F7F7F7F7F7F
    ffm = int(ffm.item())
    assert (-1 if ffm == 0x7F7F7F7F7F7F7F7F else ffm) == offm
    assert np.array_equal(m16.cpu().numpy(), exp)
    # every other byte value, one call each, at unit (b % 64), position (b % 16)
    others = [b for b in range(256) if b not in _ALPHABET]
    assert len(others) == 192
    for b in others:
        pos = 16 * (b % 64) + (b % 16)
        t = bytearray(base[0][4])
        t[pos] = b
        texts = [list(o) for o in base]
        texts[0][4] = bytes(t)
        _, _, bad = _rv(ctx, texts, W, "device")
        assert bad == 4 * nchars + pos, (b, pos)
