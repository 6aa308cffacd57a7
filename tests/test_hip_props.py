"""Property tests (hypothesis) of the HIP kernels against the C oracle on
edge-heavy raw words (0, 1, p-1, p, p+1, 2^127, 2^128-1 and uniform 128-bit
values) and random party counts -- bit-exact, through the C ABI."""
import os

import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

pytestmark = pytest.mark.gpu

from oracle import amphora_oracle as O  # noqa: E402
from oracle import coracle  # noqa: E402

P, R, RINV = O.TEST_PRIME, O.TEST_R, O.TEST_RINV
EDGE = [0, 1, 2, P - 2, P - 1, P, P + 1, 2 ** 127, 2 ** 128 - 1, 2 ** 128 - P - 1]
raw_word = st.one_of(st.sampled_from(EDGE), st.integers(0, 2 ** 128 - 1))
# AMPH_HYPOTHESIS_EXAMPLES raises the example count for soak runs
SETTINGS = settings(max_examples=int(os.environ.get("AMPH_HYPOTHESIS_EXAMPLES", "50")), deadline=None,
                    suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])


@pytest.fixture(scope="module")
def ctx():
    import torch
    assert torch.cuda.is_available()
    import amphora_amd as A
    return A.Context(P, R, RINV)


@pytest.fixture(scope="module")
def F():
    return coracle.test_field(threads=1)


def arr(vals, width=16):
    b = b"".join(int(v).to_bytes(16, "little") for v in vals)
    return np.frombuffer(b, np.uint8).reshape(-1, width).copy()


@SETTINGS
@given(st.integers(1, 5), st.integers(1, 70), st.data())
def test_recombine_verify_edges(ctx, F, n, W, data):
    vals = data.draw(st.lists(raw_word, min_size=5 * n * W, max_size=5 * n * W))
    buf = arr(vals).reshape(5, n, W, 16)
    odos = [tuple(buf[k, j] for k in range(5)) for j in range(n)]
    y, ff = ctx.recombine_verify(odos)
    oy, off = F.recombine_verify(odos)
    assert ff == off
    assert np.array_equal(y, oy)  # secrets are written for every word, verified or not


@SETTINGS
@given(st.integers(1, 60), st.data())
def test_mask_input_edges(ctx, F, W, data):
    """Honest mask ODOs (so the masked words are defined) with edge secrets."""
    odos, _ = F.synth_odos(seed=data.draw(st.integers(0, 2 ** 32)), n=2, W=W, noncanon_permille=300)
    secrets = arr(data.draw(st.lists(raw_word, min_size=W, max_size=W)))
    out, ff = ctx.mask_input(odos, secrets)
    oo, off = F.mask_input(secrets, odos)
    assert ff == off == -1 and np.array_equal(out, oo)


@SETTINGS
@given(st.integers(1, 60), raw_word, st.booleans(), st.data())
def test_convert_share_edges(ctx, F, W, key, zero, data):
    masked = arr(data.draw(st.lists(raw_word, min_size=W, max_size=W)))
    tuples = arr(data.draw(st.lists(raw_word, min_size=2 * W, max_size=2 * W)), 32)
    got = ctx.convert_share(masked, tuples, key % P, zero)
    assert np.array_equal(got, F.convert_share(masked, tuples, key % P, zero))


@SETTINGS
@given(st.integers(1, 40), st.integers(1, 4), st.integers(0, 1), st.data())
def test_odo_kernels_edges(ctx, F, W, n, p0, data):
    share = arr(data.draw(st.lists(raw_word, min_size=W, max_size=W)))
    masks = arr(data.draw(st.lists(raw_word, min_size=4 * W, max_size=4 * W)), 32)
    trip = arr(data.draw(st.lists(raw_word, min_size=12 * W, max_size=12 * W)), 96)
    got = ctx.odo_pre(share, 16, masks, trip)
    exp = F.odo_pre(share, 16, masks, trip)
    for g, e in zip(got, exp):
        assert np.array_equal(g, e)
    # partners: arbitrary signed diffs with magnitudes < p
    mags, negs = [got[3]], [got[4]]
    for _ in range(n - 1):
        mags.append(arr([v % P for v in data.draw(st.lists(raw_word, min_size=4 * W, max_size=4 * W))])
                    .reshape(2 * W, 2, 16))
        negs.append(np.array(data.draw(st.lists(st.integers(0, 1), min_size=4 * W, max_size=4 * W)),
                             np.uint8).reshape(2 * W, 2))
    opened = ctx.open_diffs(mags, negs)
    assert np.array_equal(opened, F.recombine_diffs(mags, negs))
    w, u = ctx.odo_post(opened, trip, p0 == 1)
    ew, eu = F.odo_post(opened.reshape(2 * W, 32), trip, p0 == 1)
    assert np.array_equal(w, ew) and np.array_equal(u, eu)
    w, u = ctx.open_post(mags, negs, trip, p0 == 1)
    assert np.array_equal(w, ew) and np.array_equal(u, eu)


@SETTINGS
@given(st.lists(raw_word, min_size=1, max_size=80))
def test_codec_edges(ctx, F, vals):
    a = arr(vals)
    spdz = O.MpSpdzIntegrationUtils(P, R, RINV)
    assert [int.from_bytes(x.tobytes(), "little") for x in ctx.from_gfp(a)] == \
        [spdz.from_gfp(x.tobytes()) for x in a]
    assert [x.tobytes() for x in ctx.to_gfp(a)] == [spdz.to_gfp(v % P) for v in vals]


# signed diffs as the Beaver exchange carries them: magnitudes < 2^128 with
# every decimal length and the 10^k / 2^k edges
_DEC_EDGE = sorted({v for k in range(39) for v in (10 ** k - 1, 10 ** k, 10 ** k + 1) if 0 <= v < 2 ** 128} |
                   {v for k in range(129) for v in (2 ** k - 1, 2 ** k) if v < 2 ** 128})
signed_diff = st.builds(lambda m, s: -m if s else m,
                        st.one_of(st.sampled_from(_DEC_EDGE), st.integers(0, 2 ** 128 - 1),
                                  st.integers(0, 10 ** 12)), st.booleans())


@SETTINGS
@given(st.lists(st.tuples(signed_diff, signed_diff), min_size=1, max_size=300))
def test_exchange_codec_edges(ctx, pairs):
    """MultiplicationExchangeObject interimValues: the GPU encode is byte-for-byte
    Jackson's compact text (json.dumps with BigInteger semantics: no "-0"), and
    the GPU decode of that text gives back the signed values."""
    import json
    text = json.dumps([{"a": a, "b": b} for a, b in pairs], separators=(",", ":")).encode()
    mag = np.zeros((len(pairs), 2, 16), np.uint8)
    neg = np.zeros((len(pairs), 2), np.uint8)
    for k, ab in enumerate(pairs):
        for j, x in enumerate(ab):
            mag[k, j] = np.frombuffer(abs(x).to_bytes(16, "little"), np.uint8)
            neg[k, j] = x < 0
    assert ctx.exchange_encode(mag, neg) == text
    m2, n2 = ctx.exchange_decode(text, len(pairs))
    assert np.array_equal(m2, mag) and np.array_equal(n2, neg)
