"""The reference's own tests, restated against the host-side mirror
(amphora_amd.client / amphora_amd.service), which runs every word of
arithmetic on the GPU through the C ABI.

* service SecretShareUtilTest.java:48-107        -> test_kat1_*
* OutputDeliveryServiceTest.java:211-382         -> test_kat2_*
* client SecretShareUtilTest.java:30-85          -> test_kat3_*
* DefaultAmphoraClientTest.java:193-271          -> test_roundtrip_*
"""
import json
import os
import random
import uuid

import pytest

pytestmark = pytest.mark.gpu

from oracle import amphora_oracle as O  # noqa: E402

P, R, RINV = O.TEST_PRIME, O.TEST_R, O.TEST_RINV
SPDZ = O.MpSpdzIntegrationUtils(P, R, RINV)


@pytest.fixture(scope="module")
def kat(golden_dir):
    with open(os.path.join(golden_dir, "kat.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def A():
    import torch
    assert torch.cuda.is_available()
    import amphora_amd
    return amphora_amd


@pytest.fixture(scope="module")
def client_util(A):
    from amphora_amd.client import SecretShareUtil
    return SecretShareUtil.of(P, R, RINV)


@pytest.fixture(scope="module")
def ctx(client_util):
    return client_util.context


def test_kat1_convert_to_secret_share(A, ctx, kat):
    from amphora_amd.service import SecretShareUtil
    k = kat["kat1"]
    util = SecretShareUtil(ctx)
    mac_key = int(k["mac_key"]) % P
    mi = A.MaskedInput(uuid.UUID("3bcf8308-8f50-4d24-a37b-b0075bb5e779"),
                       [A.MaskedInputData.of(SPDZ.to_gfp(int(x) % P)) for x in k["masked_inputs"]],
                       ["t"])
    masks = [(SPDZ.to_gfp(int(v) % P), SPDZ.to_gfp(int(m) % P)) for v, m in k["input_masks"]]
    share = util.convert_to_secret_share(mi, str(mac_key), masks, False)
    assert share.data == b"".join(SPDZ.to_gfp(int(x) % P) for x in k["expected_share_words"])
    assert share.secret_id == mi.secret_id and share.tags == ["t"]


def test_kat1_length_mismatch(A, ctx):
    from amphora_amd.service import SecretShareUtil
    mi = A.MaskedInput(uuid.uuid4(), [A.MaskedInputData.of(bytes(16))], [])
    with pytest.raises(A.IllegalArgumentException,
                       match="^Received more input data than available inputMasks.$"):
        SecretShareUtil(ctx).convert_to_secret_share(mi, "", [], False)


def _kat2_service(A, ctx, kat, fail_castor=False, fail_open=False):
    from amphora_amd.service import (INPUT_MASK_GFP, MULTIPLICATION_TRIPLE_GFP,
                                     OutputDeliveryService)
    k = kat["kat2"]
    masks = b"".join(SPDZ.to_gfp(v) + SPDZ.to_gfp(0) for v in k["input_mask_values"])
    triples = b"".join(SPDZ.to_gfp(a) + SPDZ.to_gfp(0) + SPDZ.to_gfp(b) + SPDZ.to_gfp(0)
                       + SPDZ.to_gfp(c) + SPDZ.to_gfp(0) for a, b, c in k["triples"])
    req, op = uuid.UUID(k["request_id"]), uuid.UUID(k["expected_operation_id"])
    calls = []

    def castor(rid, ttype, count):
        calls.append((rid, ttype, count))
        if fail_castor:
            raise IOError("No tuples")
        if ttype == INPUT_MASK_GFP:
            assert rid == req and count == 4
            return masks
        assert ttype == MULTIPLICATION_TRIPLE_GFP and rid == op and count == 4
        return triples

    def exchange(xo):
        if fail_open:
            raise IOError("Failed")
        return [[A.FactorPair(a, b) for a, b in k["partner_diffs"]]]

    return OutputDeliveryService(ctx, k["player_id"], castor, exchange), req, calls


def test_kat2_compute_output_delivery_object(A, ctx, kat):
    k = kat["kat2"]
    svc, req, _ = _kat2_service(A, ctx, kat)
    share = A.SecretShare(uuid.UUID("5decd680-bdec-4426-bcc6-376ef232e474"),
                          b"".join(SPDZ.to_gfp(v) + SPDZ.to_gfp(0) for v in k["secret_values"]))
    odo = svc.compute_output_delivery_object(share, req)
    xo = svc.last_exchange_object
    assert str(xo.operation_id) == k["expected_operation_id"] and xo.player_id == 0
    assert [[fp.a, fp.b] for fp in xo.interim_values] == k["expected_own_diffs"]
    mv, pr = k["input_mask_values"], k["expected_products"]
    expected = A.OutputDeliveryObject(b"".join(SPDZ.to_gfp(v) for v in k["secret_values"]),
                                      b"".join(SPDZ.to_gfp(v) for v in mv[0::2]),
                                      b"".join(SPDZ.to_gfp(v) for v in mv[1::2]),
                                      b"".join(SPDZ.to_gfp(v) for v in pr[0::2]),
                                      b"".join(SPDZ.to_gfp(v) for v in pr[1::2]))
    assert odo == expected


def test_kat2_json_exchange(A, ctx, kat):
    """The same KAT with the open carried as MultiplicationExchangeObject JSON
    bodies (exchange_format="json", GPU-coded)."""
    import json
    from amphora_amd.service import OutputDeliveryService
    k = kat["kat2"]
    svc0, req, _ = _kat2_service(A, ctx, kat)
    seen = []

    def exchange(body):
        seen.append(body)
        return [json.dumps({"operationId": k["expected_operation_id"], "playerId": 1,
                            "interimValues": [{"a": a, "b": b} for a, b in k["partner_diffs"]]},
                           separators=(",", ":")).encode()]

    svc = OutputDeliveryService(ctx, k["player_id"], svc0._tuples, exchange, exchange_format="json")
    share = A.SecretShare(None, b"".join(SPDZ.to_gfp(v) + SPDZ.to_gfp(0) for v in k["secret_values"]))
    odo = svc.compute_output_delivery_object(share, req)
    assert seen[0] == json.dumps({"operationId": k["expected_operation_id"], "playerId": 0,
                                  "interimValues": [{"a": a, "b": b} for a, b in k["expected_own_diffs"]]},
                                 separators=(",", ":")).encode()
    assert odo == svc0.compute_output_delivery_object(share, req)


def test_kat2_failure_messages(A, ctx, kat):
    k = kat["kat2"]
    share = A.SecretShare(None, b"".join(SPDZ.to_gfp(v) + SPDZ.to_gfp(0) for v in k["secret_values"]))
    svc, req, _ = _kat2_service(A, ctx, kat, fail_castor=True)
    with pytest.raises(A.AmphoraServiceException,
                       match="^Failed to retrieve the required Tuples form Castor$"):
        svc.compute_output_delivery_object(share, req)
    svc, req, _ = _kat2_service(A, ctx, kat, fail_open=True)
    with pytest.raises(A.AmphoraServiceException,
                       match="^Failed to open values for operation #%s$" % k["expected_operation_id"]):
        svc.compute_output_delivery_object(share, req)


def test_input_masks_as_odo(A, ctx):
    """InputMaskCachingService.getInputMasksAsOutputDeliveryObject :77-99 vs the oracle."""
    from amphora_amd.service import OutputDeliveryService
    rng = random.Random(3)
    W = 37
    mstream = b"".join(SPDZ.to_gfp(rng.randrange(P)) + SPDZ.to_gfp(rng.randrange(P)) for _ in range(W))
    odo_masks = b"".join(SPDZ.to_gfp(rng.randrange(P)) + SPDZ.to_gfp(0) for _ in range(2 * W))
    triples = b"".join(SPDZ.to_gfp(rng.randrange(P)) for _ in range(2 * W * 6))
    partner = [(rng.randrange(-P + 1, P), rng.randrange(-P + 1, P)) for _ in range(2 * W)]
    req = uuid.uuid4()
    odo_req = O.odo_request_id(req)

    def castor(rid, ttype, count):
        if rid == req:
            return mstream
        if rid == odo_req:
            return odo_masks
        return triples

    svc = OutputDeliveryService(ctx, 1, castor, lambda xo: [[A.FactorPair(a, b) for a, b in partner]])
    odo, cached = svc.get_input_masks_as_output_delivery_object(req, W)
    values16 = b"".join(mstream[32 * i:32 * i + 16] for i in range(W))
    exp, _, _ = O.compute_output_delivery_object(SPDZ, values16, odo_masks, triples, [partner], 1)
    assert cached.shape == (W, 32)
    assert all(bytes(a) == b for a, b in zip(odo.fields(), (exp.secret_shares, exp.r_shares,
                                                            exp.v_shares, exp.w_shares, exp.u_shares)))


def _abs_next_long(rng):
    return abs(rng.getrandbits(64) - 2 ** 63)


def test_kat3_verify_secrets(A, client_util):
    rng = random.Random(42)
    n = 5
    s = [_abs_next_long(rng) for _ in range(n)]
    r = [_abs_next_long(rng) for _ in range(n)]
    v = [_abs_next_long(rng) for _ in range(n)]
    w = [a * b for a, b in zip(s, r)]
    u = [a * b for a, b in zip(v, r)]
    client_util.verify_secrets(s, r, u, v, w)
    w[-1] -= 10
    with pytest.raises(A.IntegrityVerificationException) as ei:
        client_util.verify_secrets(s, r, u, v, w)
    assert str(ei.value).startswith("Verification of secret has failed")
    assert str(ei.value) == O.verification_failure_message(P, n - 1, s, r, u, v, w)


def _odos_for(rng, secrets):
    b = [[[] for _ in range(5)] for _ in range(2)]
    for s in secrets:
        r = rng.getrandbits(64) - 2 ** 63
        v = rng.getrandbits(64) - 2 ** 63
        for k, x in enumerate((s, r, v, s * r % P, v * r % P)):
            mask = rng.getrandbits(P.bit_count() - 1)
            b[0][k].append(SPDZ.to_gfp(mask))
            b[1][k].append(SPDZ.to_gfp((x - mask) % P))
    return [[b"".join(b[j][k]) for k in range(5)] for j in range(2)]


def test_roundtrip_create_secret(A, client_util):
    from amphora_amd.client import create_masked_input
    rng = random.Random(1)
    for _ in range(20):
        size = rng.randrange(1, 1000)
        secrets = [rng.randrange(2 ** 63) for _ in range(size)]
        masks = [rng.getrandbits(P.bit_length()) % P for _ in range(size)]
        odos = [A.OutputDeliveryObject(*f) for f in _odos_for(rng, masks)]
        mi = create_masked_input(client_util, A.Secret.of([], secrets), odos)
        assert len(mi.data) == size
        for j in range(size):
            m = sum(SPDZ.from_gfp(bytes(o.secret_shares[16 * j:16 * j + 16])) for o in odos) % P
            assert (m + SPDZ.from_gfp(mi.data[j].value)) % P == secrets[j]


def test_roundtrip_get_secret(A, client_util):
    from amphora_amd.client import verify_output_delivery_objects
    rng = random.Random(2)
    for _ in range(20):
        size = rng.randrange(1, 1000)
        secrets = [rng.randrange(2 ** 63) for _ in range(size)]
        odos = [A.OutputDeliveryObject(*f) for f in _odos_for(rng, secrets)]
        assert verify_output_delivery_objects(client_util, odos) == secrets


def test_get_secret_tampered_raises_reference_message(A, client_util):
    from amphora_amd.client import verify_output_delivery_objects
    rng = random.Random(5)
    secrets = [rng.randrange(2 ** 63) for _ in range(50)]
    f = _odos_for(rng, secrets)
    w1 = bytearray(f[1][3])
    w1[16 * 17] ^= 1  # corrupt party 1's w share of word 17
    f[1][3] = bytes(w1)
    odos = [A.OutputDeliveryObject(*x) for x in f]
    util = O.ClientSecretShareUtil(P, R, RINV)
    po = [O.OutputDeliveryObject(*x) for x in f]
    with pytest.raises(O.IntegrityVerificationException) as oe:
        O.verify_output_delivery_objects(util, po)
    with pytest.raises(A.IntegrityVerificationException) as ne:
        verify_output_delivery_objects(client_util, odos)
    assert str(ne.value) == str(oe.value)


def test_mask_input_single_word(A, client_util):
    for s, m in ((5, 7), (P - 1, 3), (-12, 2 ** 130 + 5)):
        got = client_util.mask_input(s, m)
        assert got.value == SPDZ.to_gfp((s - m) % P)


def test_recombine_object(client_util):
    assert client_util.recombine_object([]) == []
    one = SPDZ.to_gfp(5) + b"\x01\x02"
    assert client_util.recombine_object([one, SPDZ.to_gfp(7) + b"\x00\x00"]) == [12]


def test_create_secret_more_secrets_than_masks(A, client_util):
    """More secret words than masks: the mask ODOs are verified first
    (verifyOutputDeliveryObjects, DefaultAmphoraClient.java:153), so tampered
    masks raise IntegrityVerificationException; honest ones the index error of
    inputMasks.get(i) (:155-157)."""
    from amphora_amd.client import create_masked_input
    rng = random.Random(8)
    masks = [rng.randrange(P) for _ in range(10)]
    f = _odos_for(rng, masks)
    secret = A.Secret.of([], list(range(11)))
    with pytest.raises(IndexError):
        create_masked_input(client_util, secret, [A.OutputDeliveryObject(*x) for x in f])
    w1 = bytearray(f[1][3])
    w1[16 * 4] ^= 1
    f[1][3] = bytes(w1)
    with pytest.raises(A.IntegrityVerificationException, match="^Verification of secret has failed"):
        create_masked_input(client_util, secret, [A.OutputDeliveryObject(*x) for x in f])


def test_create_secret_json_more_secrets_than_masks(A, client_util):
    """The same order from the parties' JSON bodies (one fused wire call:
    amph_mask_input_b64 verifies before it reports the length)."""
    from amphora_amd import wire
    from amphora_amd.client import create_masked_input_json
    rng = random.Random(9)
    masks = [rng.randrange(P) for _ in range(10)]
    f = _odos_for(rng, masks)
    secret = A.Secret.of([], list(range(11)))
    bodies = [wire.odo_to_json(client_util.context, A.OutputDeliveryObject(*x)) for x in f]
    with pytest.raises(IndexError):
        create_masked_input_json(client_util, secret, bodies)
    w1 = bytearray(f[1][3])
    w1[16 * 4] ^= 1
    f[1][3] = bytes(w1)
    bodies = [wire.odo_to_json(client_util.context, A.OutputDeliveryObject(*x)) for x in f]
    with pytest.raises(A.IntegrityVerificationException, match="^Verification of secret has failed"):
        create_masked_input_json(client_util, secret, bodies)


@pytest.mark.parametrize("short", ["masks", "triples"])
def test_short_castor_stream(A, ctx, kat, short):
    """A Castor download with fewer tuples than requested is rejected before
    any kernel reads past it (the reference fails on the missing index)."""
    from amphora_amd.service import INPUT_MASK_GFP
    svc, req, _ = _kat2_service(A, ctx, kat)
    inner = svc._tuples

    def castor(rid, ttype, count):
        data = inner(rid, ttype, count)
        cut = (ttype == INPUT_MASK_GFP) == (short == "masks")
        return data[: -(32 if ttype == INPUT_MASK_GFP else 96)] if cut else data

    svc._tuples = castor
    k = kat["kat2"]
    share = A.SecretShare(None, b"".join(SPDZ.to_gfp(v) + SPDZ.to_gfp(0) for v in k["secret_values"]))
    with pytest.raises(A.AmphoraServiceException, match="tuples, 4 requested"):
        svc.compute_output_delivery_object(share, req)


@pytest.mark.parametrize("fmt", ["objects", "json"])
def test_short_partner_list(A, ctx, kat, fmt):
    """A partner that opens fewer FactorPairs than this party fails the open
    (recombineDiffs inside the open's Try, OutputDeliveryService.java:205-219)."""
    from amphora_amd.service import OutputDeliveryService
    k = kat["kat2"]
    svc0, req, _ = _kat2_service(A, ctx, kat)
    pairs = k["partner_diffs"][:-1]
    if fmt == "json":
        def exchange(body):
            return [json.dumps({"operationId": k["expected_operation_id"], "playerId": 1,
                                "interimValues": [{"a": a, "b": b} for a, b in pairs]}).encode()]
    else:
        def exchange(xo):
            return [[A.FactorPair(a, b) for a, b in pairs]]
    svc = OutputDeliveryService(ctx, 0, svc0._tuples, exchange, exchange_format=fmt)
    share = A.SecretShare(None, b"".join(SPDZ.to_gfp(v) + SPDZ.to_gfp(0) for v in k["secret_values"]))
    with pytest.raises(A.AmphoraServiceException, match="^Failed to open values for operation #"):
        svc.compute_output_delivery_object(share, req)


def test_native_length_checks(A, ctx):
    """The ctypes layer checks buffer lengths the C entry points cannot see."""
    import numpy as np
    from amphora_amd._lib import AmphoraNativeError
    z = lambda n, w=16: np.zeros((n, w), np.uint8)  # noqa: E731
    with pytest.raises(AmphoraNativeError, match="input-mask tuples"):
        ctx.odo_pre(z(4, 32), 32, z(7, 32), z(8, 96))
    with pytest.raises(AmphoraNativeError, match="multiplication triples"):
        ctx.odo_pre(z(4, 32), 32, z(8, 32), z(7, 96))
    mag, neg = np.zeros((8, 2, 16), np.uint8), np.zeros((8, 2), np.uint8)
    with pytest.raises(AmphoraNativeError, match="differ in length"):
        ctx.open_diffs([mag, mag[:7]], [neg, neg[:7]])
    with pytest.raises(AmphoraNativeError, match="do not match"):
        ctx.odo_post(mag[:6], z(8, 96), True)
    with pytest.raises(AmphoraNativeError, match="inputMasks"):
        ctx.convert_share(z(5), z(4, 32), 1, False)
    with pytest.raises(AmphoraNativeError, match="same length"):
        ctx.recombine_verify([(z(4), z(4), z(3), z(4), z(4))])
