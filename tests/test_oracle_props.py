"""Property tests (hypothesis) of the C oracle -- the checker the GPU parity
tests use at large sizes -- against the Python restatement of the reference's
BigInteger code, on edge-heavy raw words: 0, 1, p-1, p, p+1, 2^127, 2^128-1
(non-canonical words >= p occur in the reference's random-byte fixtures,
AmphoraTestData.java) and uniform 128-bit values.  CPU only."""
import os

import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from oracle import amphora_oracle as O
from oracle import coracle

P, R, RINV = O.TEST_PRIME, O.TEST_R, O.TEST_RINV
SPDZ = O.MpSpdzIntegrationUtils(P, R, RINV)
EDGE = [0, 1, 2, P - 2, P - 1, P, P + 1, 2 ** 127, 2 ** 128 - 1, 2 ** 128 - P - 1]
raw_word = st.one_of(st.sampled_from(EDGE), st.integers(0, 2 ** 128 - 1))
# AMPH_HYPOTHESIS_EXAMPLES raises the example count for soak runs
SETTINGS = settings(max_examples=int(os.environ.get("AMPH_HYPOTHESIS_EXAMPLES", "60")), deadline=None,
                    suppress_health_check=[HealthCheck.too_slow])


@pytest.fixture(scope="module")
def F():
    return coracle.test_field(threads=1)


def arr(vals):
    return np.frombuffer(b"".join(int(v).to_bytes(16, "little") for v in vals), np.uint8).reshape(-1, 16).copy()


def ints(a):
    return [int.from_bytes(a[i].tobytes(), "little") for i in range(a.shape[0])]


@SETTINGS
@given(st.integers(1, 4).flatmap(lambda n: st.lists(st.lists(raw_word, min_size=n, max_size=n),
                                                    min_size=1, max_size=12)))
def test_recombine(F, rows):
    n = len(rows[0])
    shares = [arr([r[j] for r in rows]) for j in range(n)]
    util = O.ClientSecretShareUtil(P, R, RINV)
    assert ints(F.recombine(shares)) == util.recombine_object([s.tobytes() for s in shares])


@SETTINGS
@given(st.lists(st.tuples(raw_word, raw_word, raw_word, raw_word, raw_word), min_size=1, max_size=10),
       st.data())
def test_recombine_verify_single_party(F, words, data):
    """One party holding (y, r, v, w, u) raw; w/u made consistent or not."""
    fix = data.draw(st.lists(st.booleans(), min_size=len(words), max_size=len(words)))
    cols = [list(c) for c in zip(*words)]
    for i, ok in enumerate(fix):
        if ok:  # w = y r, u = v r in the Montgomery domain
            y, r, v = (SPDZ.from_gfp(int(cols[k][i]).to_bytes(16, "little")) for k in range(3))
            cols[3][i] = int.from_bytes(SPDZ.to_gfp(y * r % P), "little")
            cols[4][i] = int.from_bytes(SPDZ.to_gfp(v * r % P), "little")
    odo = tuple(arr(c) for c in cols)
    y, ff = F.recombine_verify([odo])
    po = O.OutputDeliveryObject(*[a.tobytes() for a in odo])
    util = O.ClientSecretShareUtil(P, R, RINV)
    try:
        exp = O.verify_output_delivery_objects(util, [po])
        assert ff == -1 and ints(y) == exp
    except O.IntegrityVerificationException:
        ys = util.recombine_object([odo[0].tobytes()])
        rs = util.recombine_object([odo[1].tobytes()])
        vs = util.recombine_object([odo[2].tobytes()])
        ws = util.recombine_object([odo[3].tobytes()])
        us = util.recombine_object([odo[4].tobytes()])
        assert ff == O.first_failing_index(P, ys, rs, us, vs, ws)


@SETTINGS
@given(st.lists(st.tuples(raw_word, raw_word, raw_word), min_size=1, max_size=10), raw_word,
       st.booleans())
def test_convert_share(F, rows, key, zero):
    masked = arr([r[0] for r in rows])
    tuples = np.concatenate([arr([r[1] for r in rows]), arr([r[2] for r in rows])], axis=1).copy()
    got = F.convert_share(masked, tuples, key, zero)
    exp = O.convert_to_secret_share(SPDZ, [masked[i].tobytes() for i in range(len(rows))], str(key % P),
                                    [(tuples[i, :16].tobytes(), tuples[i, 16:].tobytes()) for i in range(len(rows))],
                                    zero)
    assert got.tobytes() == exp


@SETTINGS
@given(st.lists(st.tuples(*[raw_word] * 9), min_size=1, max_size=6),
       st.lists(st.tuples(st.integers(-P + 1, P - 1), st.integers(-P + 1, P - 1)), min_size=12,
                max_size=12),
       st.integers(0, 2))
def test_output_delivery_object(F, rows, partner, player):
    """K_ODO_PRE -> open -> K_ODO_POST restated in C vs the Python
    computeOutputDeliveryObject, one partner with arbitrary signed diffs."""
    W = len(rows)
    share16 = arr([r[0] for r in rows])
    masks = arr([x for r in rows for x in (r[1], 0, r[2], 0)]).reshape(2 * W, 32)
    trip = arr([x for r in rows for x in (r[3], 0, r[4], 0, r[5], 0, r[6], 0, r[7], 0, r[8], 0)]).reshape(2 * W, 96)
    y, r, v, mag, neg = F.odo_pre(share16, 16, masks, trip)
    pdiffs = partner[:2 * W]
    pm = arr([abs(x) for d in pdiffs for x in d]).reshape(2 * W, 2, 16)
    pn = np.array([[d[0] < 0, d[1] < 0] for d in pdiffs], np.uint8)
    opened = F.recombine_diffs([mag, pm], [neg, pn])
    w, u = F.odo_post(opened.reshape(2 * W, 32), trip, player == 0)
    exp, own, _ = O.compute_output_delivery_object(SPDZ, share16.tobytes(), masks.tobytes(), trip.tobytes(),
                                                   [pdiffs], player)
    assert y.tobytes() == exp.secret_shares and r.tobytes() == exp.r_shares and v.tobytes() == exp.v_shares
    assert w.tobytes() == exp.w_shares and u.tobytes() == exp.u_shares
    got_own = [(-a if na else a, -b if nb else b) for (a, b), (na, nb) in
               zip([(ints(mag[k:k + 1, 0])[0], ints(mag[k:k + 1, 1])[0]) for k in range(2 * W)], neg.tolist())]
    assert got_own == own
