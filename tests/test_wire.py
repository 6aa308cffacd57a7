"""Wire codec (GPU base64 + JSON framing) against the reference's JSON test
and Python's standard base64 module.

* amphora-common/.../entities/VerifiableSecretTest.java:25-100 -- exact pretty
  JSON of a VerifiableSecretShare, parse back, missing-field error message.
* base64: Jackson writes byte[] with Base64Variants.MIME_NO_LINEFEEDS
  (standard alphabet, '=' padding, no line breaks) == Python's b64encode.
"""
import base64
import json
import random
import uuid

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from oracle import amphora_oracle as O  # noqa: E402

P, R, RINV = O.TEST_PRIME, O.TEST_R, O.TEST_RINV


@pytest.fixture(scope="module")
def ctx():
    import torch
    assert torch.cuda.is_available()
    import amphora_amd as A
    return A.Context(P, R, RINV)


def _vss_expected():
    # VerifiableSecretTest.java:26-69, assembled from the same parts
    sid = "80fbba1b-3da8-4b1e-8a2c-cebd65229fad"
    b = {k: base64.b64encode(v).decode() for k, v in
         (("s", b"sShares"), ("r", b"rShares"), ("v", b"vShares"), ("w", b"wShares"), ("u", b"uShares"))}
    return ("{\n"
            '  "secretId" : "' + sid + '",\n'
            '  "tags" : [ {\n'
            '    "key" : "carbyne",\n'
            '    "value" : "stack",\n'
            '    "valueType" : "STRING"\n'
            "  } ],\n"
            '  "secretShares" : "' + b["s"] + '",\n'
            '  "rShares" : "' + b["r"] + '",\n'
            '  "vShares" : "' + b["v"] + '",\n'
            '  "wShares" : "' + b["w"] + '",\n'
            '  "uShares" : "' + b["u"] + '"\n'
            "}")


def test_vss_json_matches_reference(ctx):
    import amphora_amd as A
    from amphora_amd import wire
    odo = A.OutputDeliveryObject(b"sShares", b"rShares", b"vShares", b"wShares", b"uShares")
    sid = uuid.UUID("80fbba1b-3da8-4b1e-8a2c-cebd65229fad")
    tags = [{"key": "carbyne", "value": "stack"}]
    text = wire.vss_to_json(ctx, sid, tags, odo, pretty=True)
    assert text == _vss_expected()
    sid2, tags2, odo2 = wire.vss_from_json(ctx, _vss_expected())
    assert sid2 == sid and odo2 == odo
    assert tags2 == [{"key": "carbyne", "value": "stack", "valueType": "STRING"}]
    # compact form parses back to the same object
    assert wire.vss_from_json(ctx, wire.vss_to_json(ctx, sid, tags, odo, pretty=False))[2] == odo


def test_vss_json_missing_field(ctx):
    import re
    import amphora_amd as A
    from amphora_amd import wire
    invalid = re.sub(r'"rShares" :\s"\S+",', "", _vss_expected(), count=1)
    with pytest.raises(A.IllegalArgumentException, match="rShares is marked non-null but is null"):
        wire.vss_from_json(ctx, invalid)


@pytest.mark.parametrize("mode", ["host", "device"])
def test_base64_roundtrip_lengths(ctx, mode):
    import torch
    rng = random.Random(1)
    for n in list(range(0, 40)) + [1000, 4097, 100_003]:
        raw = bytes(rng.getrandbits(8) for _ in range(n)) if n < 5000 else np.random.default_rng(n).integers(
            0, 256, n, dtype=np.uint8).tobytes()
        exp = base64.b64encode(raw)
        if mode == "host":
            assert ctx.base64_encode(raw) == exp, n
            assert ctx.base64_decode(exp) == raw, n
        else:
            t = torch.frombuffer(bytearray(raw), dtype=torch.uint8).cuda() if n else torch.empty(0, dtype=torch.uint8, device="cuda")
            enc = ctx.base64_encode(t)
            assert enc.cpu().numpy().tobytes() == exp, n
            if n:
                dec, bad = ctx.base64_decode(enc)
                assert dec.cpu().numpy().tobytes() == raw and int(bad.item()) == 0x7F7F7F7F7F7F7F7F, n


def test_base64_host_batches_and_large(ctx):
    raw = np.random.default_rng(7).integers(0, 256, 12 * 50_000 + 5, dtype=np.uint8).tobytes()
    ctx.set_batch_words(4096)  # many batches through the 3-slot pipeline
    try:
        enc = ctx.base64_encode(raw)
        dec = ctx.base64_decode(enc)
    finally:
        ctx.set_batch_words(4 << 20)
    assert enc == base64.b64encode(raw) and dec == raw


def test_base64_invalid(ctx):
    good = base64.b64encode(bytes(range(200)))
    with pytest.raises(ValueError, match="multiple of 4"):
        ctx.base64_decode(good[:-1])
    bad = bytearray(good)
    bad[77] = ord("*")
    with pytest.raises(ValueError, match="index 77"):
        ctx.base64_decode(bytes(bad))
    bad = bytearray(good)
    bad[10] = ord("=")  # padding in the middle
    with pytest.raises(ValueError, match="index 10"):
        ctx.base64_decode(bytes(bad))


def test_base64_words(ctx):
    rng = np.random.default_rng(3)
    words = rng.integers(0, 256, (10_001, 16), dtype=np.uint8)
    rec = ctx.base64_encode_words(words)
    exp = [base64.b64encode(w.tobytes()) for w in words[:300]]
    assert [r.tobytes() for r in rec[:300]] == exp
    assert np.array_equal(ctx.base64_decode_words(rec), words)
    bad = rec.copy()
    bad[4242, 3] = ord("!")
    with pytest.raises(ValueError, match="4242"):
        ctx.base64_decode_words(bad)


def test_masked_input_json_roundtrip(ctx):
    import amphora_amd as A
    from amphora_amd import wire
    rng = np.random.default_rng(4)
    data = [A.MaskedInputData.of(rng.integers(0, 256, 16, dtype=np.uint8).tobytes()) for _ in range(5000)]
    mi = A.MaskedInput(uuid.uuid4(), data, [{"key": "k", "value": "v"}])
    text = wire.masked_input_to_json(ctx, mi)
    obj = json.loads(text)  # valid JSON, reference layout
    assert list(obj) == ["secretId", "data", "tags"]
    assert obj["data"][17] == {"value": base64.b64encode(data[17].value).decode()}
    back = wire.masked_input_from_json(ctx, text)
    assert back.secret_id == mi.secret_id and back.data == data
    with pytest.raises(A.IllegalArgumentException, match="has to be 16 bytes"):
        wire.masked_input_from_json(ctx, '{"secretId":"%s","data":[{"value":"%s"}],"tags":[]}'
                                    % (uuid.uuid4(), base64.b64encode(b"short").decode()))


def test_large_odo_json_roundtrip(ctx):
    import amphora_amd as A
    from amphora_amd import wire
    W = 200_000
    rng = np.random.default_rng(5)
    odo = A.OutputDeliveryObject(*[rng.integers(0, 256, 16 * W, dtype=np.uint8).tobytes() for _ in range(5)])
    sid = uuid.uuid4()
    text = wire.vss_to_json(ctx, sid, [], odo, pretty=False)
    sid2, tags, odo2 = wire.vss_from_json(ctx, text)
    assert sid2 == sid and tags == [] and odo2 == odo
    assert json.loads(text)["secretShares"] == base64.b64encode(bytes(odo.secret_shares)).decode()
