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
    # VerifiableSecretTest.java:102-111: the Metadata side
    invalid = re.sub(r'"secretId" :\s"\S+",', "", _vss_expected(), count=1)
    with pytest.raises(A.IllegalArgumentException, match="secretId is marked non-null but is null"):
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
                # fully asynchronous (no padding read-back): the kernel sizes the output
                dec2, bad2 = ctx.base64_decode(enc, n)
                assert dec2.cpu().numpy().tobytes() == raw and int(bad2.item()) == 0x7F7F7F7F7F7F7F7F, n
                with pytest.raises(ValueError, match="does not fit"):
                    ctx.base64_decode(enc, n + 3)


def test_base64_decode_async_reports_bad_characters(ctx):
    """The no-read-back device decode reports an illegal character (and '='
    before the padding) at its index like the synchronous form; a clean
    padded text writes no byte past its decoded length."""
    import torch
    for n in (200, 201, 202, 12 * 300):
        raw = bytes(range(256)) * (n // 256 + 1)
        raw = raw[:n]
        good = base64.b64encode(raw)
        for pos, ch in ((77, ord("*")), (10, ord("=")), (len(good) - 5, 0x80)):
            t = bytearray(good)
            t[pos] = ch
            d = torch.frombuffer(t, dtype=torch.uint8).cuda()
            _, bad = ctx.base64_decode(d, n)
            assert int(bad.item()) == pos, (n, pos)
        d = torch.frombuffer(bytearray(good), dtype=torch.uint8).cuda()
        out = torch.full((3 * len(good) // 4,), 0xEE, dtype=torch.uint8, device="cuda")
        import ctypes as C
        import amphora_amd as A
        bad = torch.full((1,), 0, dtype=torch.int64, device="cuda")
        st = A._lib.lib.amph_base64_decode(ctx._h, d.data_ptr(), len(good), out.data_ptr(), None,
                                           C.cast(C.c_void_p(bad.data_ptr()), C.POINTER(C.c_int64)),
                                           A._lib.AMPH_F_DEVICE, C.c_void_p(torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
        assert st == 0 and int(bad.item()) == 0x7F7F7F7F7F7F7F7F
        o = out.cpu().numpy().tobytes()
        assert o[:n] == raw and set(o[n:]) <= {0xEE}, n


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


_B64_ALPHABET = set(b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/")


def test_base64_block_path_every_byte_value(ctx):
    """The workgroup-staged stream decoder (full 4096-char blocks) on every
    byte value at an interior position: alphabet bytes decode like Python's
    base64, anything else is reported at its index; with two bad bytes the
    first one is reported."""
    raw = np.random.default_rng(11).integers(0, 256, 3 * 4096 * 3, dtype=np.uint8).tobytes()
    enc = base64.b64encode(raw)
    assert len(enc) % 4096 == 0
    for b in range(256):
        pos = 4096 + 13 * b + (b % 4)
        t = bytearray(enc)
        t[pos] = b
        if b in _B64_ALPHABET:
            assert ctx.base64_decode(bytes(t)) == base64.b64decode(bytes(t))
        else:
            with pytest.raises(ValueError, match="index %d$" % pos):
                ctx.base64_decode(bytes(t))
    t = bytearray(enc)
    t[9001] = ord("-")
    t[5003] = ord("_")
    with pytest.raises(ValueError, match="index 5003$"):
        ctx.base64_decode(bytes(t))


def test_base64_words_every_byte_value(ctx):
    """Per-word records: every byte value in every data position of a record."""
    words = np.random.default_rng(12).integers(0, 256, (4096, 16), dtype=np.uint8)
    rec = ctx.base64_encode_words(words)
    for b in range(256):
        bad = rec.copy()
        k = 1000 + b
        bad[k, b % 22] = b
        if b in _B64_ALPHABET:
            got = ctx.base64_decode_words(bad)
            assert got[k].tobytes() == base64.b64decode(bad[k].tobytes())
        else:
            with pytest.raises(ValueError, match=str(k)):
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


# ---- MultiplicationExchangeObject (Beaver open) ---------------------------------
def _jackson(op, pid, pairs):
    # Jackson's default (compact, declaration order) == json.dumps compact
    return json.dumps({"operationId": str(op), "playerId": pid,
                       "interimValues": [{"a": a, "b": b} for a, b in pairs]},
                      separators=(",", ":")).encode()


def _diff_arrays(pairs):
    mag = np.zeros((len(pairs), 2, 16), np.uint8)
    neg = np.zeros((len(pairs), 2), np.uint8)
    for k, ab in enumerate(pairs):
        for j, x in enumerate(ab):
            mag[k, j] = np.frombuffer(abs(x).to_bytes(16, "little"), np.uint8)
            neg[k, j] = x < 0
    return mag, neg


def _random_pairs(n, seed):
    rng = random.Random(seed)
    special = [0, 1, -1, 9, -10, 10 ** 9 - 1, 10 ** 9, -(10 ** 18), 10 ** 38, -(10 ** 38) + 1,
               2 ** 128 - 1, -(2 ** 128 - 1), P - 1, -(P - 1), 2 ** 64, -(2 ** 96)]
    vals = special + [rng.choice([1, -1]) * rng.randrange(P >> rng.randrange(128)) for _ in range(2 * n)]
    vals = vals[:2 * n]
    return [(vals[2 * k], vals[2 * k + 1]) for k in range(n)]


def test_exchange_kat2_diffs(ctx):
    """OutputDeliveryServiceTest.java:64-175 own diffs, as the JSON body."""
    from amphora_amd import wire
    pairs = [(10, 25), (39, 24), (1, 148), (294, 377)]
    op = uuid.UUID("8065e700-9f48-36ba-ae8c-f881b28a28ef")
    mag, neg = _diff_arrays(pairs)
    body = wire.exchange_to_json(ctx, op, 0, mag, neg)
    assert body == (b'{"operationId":"8065e700-9f48-36ba-ae8c-f881b28a28ef","playerId":0,'
                    b'"interimValues":[{"a":10,"b":25},{"a":39,"b":24},{"a":1,"b":148},{"a":294,"b":377}]}')
    op2, pid, m2, n2 = wire.exchange_from_json(ctx, body, 4)
    assert op2 == op and pid == 0 and np.array_equal(m2, mag) and np.array_equal(n2, neg)


@pytest.mark.parametrize("n", [1, 2, 255, 256, 257, 5000, 100_003])
def test_exchange_encode_matches_jackson(ctx, n):
    from amphora_amd import wire
    pairs = _random_pairs(n, n)
    mag, neg = _diff_arrays(pairs)
    neg[0, 0] = 1 if pairs[0][0] == 0 else neg[0, 0]  # a "negative zero" prints as 0
    op = uuid.uuid4()
    body = wire.exchange_to_json(ctx, op, 3, mag, neg)
    assert body == _jackson(op, 3, pairs)
    _, _, m2, n2 = wire.exchange_from_json(ctx, body, n)
    assert np.array_equal(m2, mag)
    neg_exp = neg.copy()
    neg_exp[(mag == 0).all(axis=2)] = 0
    assert np.array_equal(n2, neg_exp)


def test_exchange_host_calls_from_two_contexts_at_once(ctx):
    """Two parties' contexts on one GPU coding their opens at the same time
    (the loopback's party threads; ctypes drops the GIL): every text and
    every decode stays exact.  With stream-ordered (hipMallocAsync) staging
    the two calls once received overlapping buffers (empty / overwritten
    texts in tools/c1_native)."""
    import threading
    import amphora_amd as A
    from amphora_amd import wire
    ctxs = [ctx, A.Context(P, R, RINV)]
    jobs = []
    for j in range(2):
        pairs = _random_pairs(8192 + 37 * j, 50 + j)
        mag, neg = _diff_arrays(pairs)
        jobs.append((mag, neg, _jackson(uuid.UUID(int=j), j, pairs)))
    errors = []

    def party(j):
        mag, neg, expect = jobs[j]
        try:
            for _ in range(30):
                body = wire.exchange_to_json(ctxs[j], uuid.UUID(int=j), j, mag, neg)
                assert body == expect
                _, _, m2, _ = wire.exchange_from_json(ctxs[j], body, mag.shape[0])
                assert np.array_equal(m2, mag)
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append((j, repr(e)[:300]))

    th = [threading.Thread(target=party, args=(j,)) for j in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors


def test_exchange_device_mode(ctx):
    import torch
    from amphora_amd import wire
    pairs = _random_pairs(20_000, 1)
    mag, neg = _diff_arrays(pairs)
    out, ln = ctx.exchange_encode(torch.from_numpy(mag).cuda(), torch.from_numpy(neg).cuda())
    arr = out[: int(ln.item())]
    assert arr.cpu().numpy().tobytes() == _jackson(uuid.UUID(int=0), 0, pairs)[
        len(b'{"operationId":"00000000-0000-0000-0000-000000000000","playerId":0,"interimValues":'):-1]
    m2, n2, bad = ctx.exchange_decode(arr, 20_000)
    assert int(bad.item()) == NO_FAIL_WORD
    assert np.array_equal(m2.cpu().numpy(), mag) and np.array_equal(n2.cpu().numpy(), neg)
    # misaligned device text (a slice at an odd offset) parses the same
    pad = torch.cat([torch.zeros(3, dtype=torch.uint8, device="cuda"), arr])[3:]
    m3, _, bad = ctx.exchange_decode(pad, 20_000)
    assert int(bad.item()) == NO_FAIL_WORD and np.array_equal(m3.cpu().numpy(), mag)


NO_FAIL_WORD = 0x7F7F7F7F7F7F7F7F


def test_exchange_decode_whitespace_and_order(ctx):
    """Any JSON writer's layout: pretty printing, members in either order."""
    pairs = _random_pairs(3000, 2)
    mag, neg = _diff_arrays(pairs)
    items = [{"b": b, "a": a} if k % 3 == 0 else {"a": a, "b": b} for k, (a, b) in enumerate(pairs)]
    text = json.dumps(items, indent=2).encode()
    m2, n2 = ctx.exchange_decode(text, 3000)
    assert np.array_equal(m2, mag)
    assert np.array_equal(n2, neg)
    text = json.dumps(items, separators=(" , ", " : ")).encode()
    m3, _ = ctx.exchange_decode(b"  \n" + text + b"\n", 3000)
    assert np.array_equal(m3, mag)
    # compact (the fast path) with members in either order
    text = json.dumps(items, separators=(",", ":")).encode()
    m4, n4 = ctx.exchange_decode(text, 3000)
    assert np.array_equal(m4, mag)
    assert np.array_equal(n4, neg)


_JSON_BUT_NOT_FACTORPAIRS = {
    b'[{"a":1,"b":2},{"a":1.5,"b":2}]', b'[{"a":1,"b":2},{"a":1e5,"b":2}]',
    b'[{"a":1,"b":2},{"a":1,"a":2}]', b'[{"a":1,"b":2},{"a":1,"c":2}]',
    b'[{"a":1,"b":2},{"a":"1","b":2}]', b'[{"a":1,"b":2},{"a":1,"b":2,"a":3}]',
    b'[{"a":1,"b":2},{"a":340282366920938463463374607431768211456,"b":2}]',
}


@pytest.mark.parametrize("text,where", [
    (b'[{"a":1,"b":2},{"a":1.5,"b":2}]', 20),
    (b'[{"a":1,"b":2},{"a":1e5,"b":2}]', 20),
    (b'[{"a":1,"b":2},{"a":1,"a":2}]', 26),
    (b'[{"a":1,"b":2},{"a":1,"c":2}]', 26),
    (b'[{"a":1,"b":2},{"a":"1","b":2}]', 20),   # values are found by their colons
    (b'[{"a":1,"b":2},{"a":1,"b":2,"a":3}]', 26),
    (b'[{"a":1,"b":2} {"a":1,"b":2}]', 20),
    (b'[{"a":1,"b":2},{"a":340282366920938463463374607431768211456,"b":2}]', 20),
    (b'[{"a":1,"b":2},{"a":--1,"b":2}]', 20),
    (b'[{"a":1,"b":2},{"a":01,"b":2}]', 20),   # leading zero (Jackson's default rejects it)
    (b'[{"a":1,"b":2},{"a":-00,"b":2}]', 20),
    (b'[{"a":1,"b":2}x,{"a":1,"b":2}]', 21),    # bytes between objects
    (b'[{"a":1,"b":2}}, {"a":1,"b":2}]', 22),
    (b'[{"a":1,"b":2},,{"a":1,"b":2}]', 21),
    (b'[{"a":1,"b":2},{"a":1,"b":2}x]', 26),    # bytes before the closing bracket
    (b'[{"a":1,"b":2},{"a":1,"b":2}]]', 26),
    (b'[{"a":1,"b":2},{"a":1,"b":2}] [', 26),   # bytes after the array
])
def test_exchange_decode_rejects(ctx, text, where):
    """Every byte of the array is checked against the FactorPair grammar; the
    reported offset is the number whose surroundings break it.  Texts that are
    not JSON at all are rejected by Python's json module too (standing in for
    Jackson); the rest are JSON but not a FactorPair list of integers."""
    try:
        json.loads(text)
        grammar_ok = True
    except ValueError:
        grammar_ok = False
    assert grammar_ok == (text in _JSON_BUT_NOT_FACTORPAIRS)
    with pytest.raises(ValueError, match="offset %d$" % where):
        ctx.exchange_decode(text, 2)


@pytest.mark.parametrize("middle,where", [
    (b'{"a":1.5,"b":2}', 20), (b'{"a":1e5,"b":2}', 20), (b'{"a":1,"a":2}', 26),
    (b'{"a":1,"c":2}', 26), (b'{"a":"1","b":2}', 20),
    (b'{"a":340282366920938463463374607431768211456,"b":2}', 20),
    (b'{"a":--1,"b":2}', 20), (b'{"a":01,"b":2}', 20), (b'{"a":-00,"b":2}', 20),
    (b'{"a":1,"b":-}', 26), (b'{"a":1,"b":2 }', 26), (b'{"a": 1,"b":2}', 21),
    (b'{"a":1,7,"b":2}', 28),    # a stray value between the members: reported at member 1
    (b'{"a":1,"b":2}5}', 36),    # stray bytes after a pair: reported at the next member 0
])
def test_exchange_decode_rejects_mid_array(ctx, middle, where):
    """The same defects in a pair that is neither first nor last, among
    compact pairs (so the numbers around it take the whitespace-free fast
    path): the same offset is reported, or none for valid whitespace."""
    text = b'[{"a":1,"b":2},' + middle + b',{"a":7,"b":8},{"a":-9,"b":10}]'
    try:
        items = json.loads(text)
        valid = all(sorted(d) == ["a", "b"] and all(type(v) is int for v in d.values())
                    and all(abs(v) < 2 ** 128 for v in d.values()) for d in items)
    except ValueError:
        valid = False
    if valid:
        mag, neg = ctx.exchange_decode(text, 4)
        exp_m, exp_n = _diff_arrays([(d["a"], d["b"]) for d in items])
        assert np.array_equal(mag, exp_m) and np.array_equal(neg, exp_n)
    else:
        with pytest.raises(ValueError, match="offset %d$" % where):
            ctx.exchange_decode(text, 4)


@pytest.mark.parametrize("text,npairs,where", [
    (b'[x{"a":1,"b":2}]', 1, 7),
    (b'x[{"a":1,"b":2}]', 1, 0),
    (b'[{"a":1,"b":2}x]', 1, 12),
    (b'[ x ]', 0, 2),
    (b'[,]', 0, 1),
])
def test_exchange_decode_rejects_edges(ctx, text, npairs, where):
    with pytest.raises(ValueError):
        json.loads(text)
    with pytest.raises(ValueError, match="offset %d$" % where):
        ctx.exchange_decode(text, npairs)


def test_exchange_decode_stray_bytes_between_pairs(ctx):
    """'...,"b":4}5},{"a":6,...': the digit before the '}' that member 0
    sees is not the previous value's, so the values around it are tied: the
    previous value's digits must end right at that '}'.  Reported at the next
    member 0, including where the two values fall in different 8 KiB decode
    spans (the tie then walks back into the previous span)."""
    pairs = _random_pairs(3000, 11)
    items = ['{"a":%d,"b":%d}' % p for p in pairs]
    ends, start = [], 1  # start: offset of item k
    for k in range(len(items) - 1):
        where = start + len(items[k]) + len('5},{"a":')  # the next member 0's number
        ycolon = start + len('{"a":%d,"b":' % pairs[k][0]) - 1  # the previous value's colon
        ends.append((k, where, ycolon))
        start += len(items[k]) + 1
    crossing = [(k, w) for k, w, y in ends if (w - 1) // 8192 != y // 8192][:4]
    ends = [(k, w) for k, w, y in ends]
    assert len(crossing) >= 2
    for k, where in crossing + [(0, ends[0][1]), (1500, ends[1500][1]), ends[-1]]:
        bad_items = list(items)
        bad_items[k] += "5}"
        text = ("[" + ",".join(bad_items) + "]").encode()
        with pytest.raises(ValueError):
            json.loads(text)
        with pytest.raises(ValueError, match="offset %d$" % where):
            ctx.exchange_decode(text, len(pairs))


def _factor_pairs_or_none(text: bytes, npairs: int):
    """The grammar oracle for the mutation test: Python's json module (any
    JSON whitespace, no trailing data) plus the FactorPair shape -- exactly
    the two members "a" and "b" per object, integer values below 2^128 in
    magnitude, npairs objects.  Returns the (a, b) list or None."""
    try:
        items = json.loads(text, object_pairs_hook=lambda kv: ("obj", kv))
    except (ValueError, UnicodeDecodeError):
        return None
    if not isinstance(items, list) or len(items) != npairs:
        return None
    out = []
    for it in items:
        if not (isinstance(it, tuple) and it[0] == "obj"):
            return None
        kv = it[1]
        if sorted(k for k, _ in kv) != ["a", "b"]:
            return None
        if any(type(v) is not int or abs(v) >= 2 ** 128 for _, v in kv):
            return None
        d = dict(kv)
        out.append((d["a"], d["b"]))
    return out


@pytest.mark.parametrize("npairs,seed,cases", [(40, 3, 2000), (700, 4, 400)])
def test_exchange_decode_mutations(ctx, npairs, seed, cases):
    """Single-byte replacements, insertions and deletions anywhere in a
    compact FactorPair array (one decode span, and several): the decoder
    accepts exactly the texts the grammar oracle accepts -- whichever of its
    passes (compact or general) takes them -- and decodes them to the
    oracle's values."""
    rng = random.Random(seed)
    pairs = _random_pairs(npairs, seed)
    base = json.dumps([{"a": a, "b": b} for a, b in pairs], separators=(",", ":")).encode()
    alphabet = b'{}[],:"ab-0123456789 x\n'
    accepted = rejected = 0
    for _ in range(cases):
        t = bytearray(base)
        i = rng.randrange(len(t) + 1)
        op = rng.randrange(3)
        c = alphabet[rng.randrange(len(alphabet))]
        if op == 0 and i < len(t):
            t[i] = c
        elif op == 1:
            t.insert(i, c)
        elif i < len(t):
            del t[i]
        text = bytes(t)
        want = _factor_pairs_or_none(text, npairs)
        if want is None:
            with pytest.raises(ValueError):
                ctx.exchange_decode(text, npairs)
            rejected += 1
        else:
            mag, neg = ctx.exchange_decode(text, npairs)
            exp_m, exp_n = _diff_arrays(want)
            assert np.array_equal(mag, exp_m) and np.array_equal(neg, exp_n), text[max(0, i - 20):i + 20]
            accepted += 1
    assert accepted > cases // 10 and rejected > cases // 3


def test_exchange_decode_block_boundaries(ctx):
    """Numbers and their keys straddling the 16 KiB workgroup spans, long
    whitespace runs longer than the staged window, "-0" and zeros."""
    pairs = _random_pairs(4000, 7)
    pairs[5] = (0, -0)
    items = ["{%s\"a\"%s:%s%d%s,%s\"b\":%d}" % (" " * (k % 7), "\n" * (k % 3), " " * (k % 5),
                                                a, " " * (k % 2), " " * (300 if k % 97 == 0 else 0), b)
             for k, (a, b) in enumerate(pairs)]
    text = ("[" + " " * 1000 + ",".join(items) + "\t" * 700 + "]").encode()
    assert [tuple(d.values()) for d in json.loads(text)] == pairs
    mag, neg = _diff_arrays(pairs)
    for off in (0, 1, 5):  # shift every number across the span boundaries
        m2, n2 = ctx.exchange_decode(b" " * off + text, len(pairs))
        assert np.array_equal(m2, mag)
        neg_exp = neg.copy()
        neg_exp[(mag == 0).all(axis=2)] = 0
        assert np.array_equal(n2, neg_exp)


def test_exchange_decode_every_length_and_the_2_128_edge(ctx):
    """The compact pass's number boundaries: every digit count 1..39 at its
    smallest and largest value (the largest 39-digit one is 2^128 - 1), both
    signs, at shifted offsets (the 8-digit chunk and span boundaries move);
    then 2^128 and a 40-digit value must be rejected where a compact text
    holds them (Jackson reads BigInteger, the field word is 128 bits)."""
    vals = []
    for L in range(1, 40):
        lo, hi = 10 ** (L - 1) if L > 1 else 0, min(10 ** L - 1, 2 ** 128 - 1)
        vals += [lo, -hi, hi, -lo if lo else 0]
    pairs = [(vals[2 * k], vals[2 * k + 1]) for k in range(len(vals) // 2)] * 40  # ~3 k pairs, several spans
    text = json.dumps([{"a": a, "b": b} for a, b in pairs], separators=(",", ":")).encode()
    mag, neg = _diff_arrays(pairs)
    assert ctx.exchange_encode(mag, neg) == text  # the formatter at every length too
    for off in (0, 3, 7):
        m2, n2 = ctx.exchange_decode(b" " * off + text, len(pairs))
        assert np.array_equal(m2, mag)
        neg_exp = neg.copy()
        neg_exp[(mag == 0).all(axis=2)] = 0
        assert np.array_equal(n2, neg_exp)
    for bad in (2 ** 128, -(2 ** 128), 10 ** 39, 2 ** 129):
        p2 = list(pairs)
        p2[len(p2) // 2] = (bad, 1)
        t2 = json.dumps([{"a": a, "b": b} for a, b in p2], separators=(",", ":")).encode()
        with pytest.raises(ValueError, match="offset"):
            ctx.exchange_decode(t2, len(p2))


def test_exchange_decode_dense_spans(ctx):
    """The count pass's colon list: spans of one-digit values ({"a":1,"b":2},
    14 bytes a pair: ~1170 values per 8 KiB span, past the list's 256-entry
    head) next to spans of long ones, at shifted offsets; then a run of
    colons (more than a span can list) is rejected."""
    rng = np.random.default_rng(17)
    pairs = []
    for blk in range(12):  # alternating dense and sparse stretches
        n = 1500 if blk % 2 == 0 else 300
        big = blk % 2 == 1
        for _ in range(n):
            a, b = (int(x) for x in rng.integers(-9, 10, 2)) if not big else \
                (int(rng.integers(0, 2 ** 62)) * 2 ** 64 - 5, -int(rng.integers(0, 2 ** 63)))
            pairs.append((a, b))
    text = json.dumps([{"a": a, "b": b} for a, b in pairs], separators=(",", ":")).encode()
    mag, neg = _diff_arrays(pairs)
    neg_exp = neg.copy()
    neg_exp[(mag == 0).all(axis=2)] = 0
    for off in (0, 1, 9):
        m2, n2 = ctx.exchange_decode(b" " * off + text, len(pairs))
        assert np.array_equal(m2, mag)
        assert np.array_equal(n2, neg_exp)
    cut = text.index(b"},", len(text) // 2) + 1
    flood = text[:cut] + b":" * 9000 + text[cut:]
    with pytest.raises(ValueError, match="offset"):
        ctx.exchange_decode(flood, len(pairs))


def test_exchange_decode_count_and_brackets(ctx):
    with pytest.raises(ValueError, match="exactly 3 FactorPairs"):
        ctx.exchange_decode(b'[{"a":1,"b":2},{"a":3,"b":4}]', 3)
    with pytest.raises(ValueError, match="offset"):
        ctx.exchange_decode(b'{"a":1,"b":2},{"a":3,"b":4}]', 2)
    m, n = ctx.exchange_decode(b"[]", 0)
    assert m.shape == (0, 2, 16)
    assert ctx.exchange_encode(np.zeros((0, 2, 16), np.uint8), np.zeros((0, 2), np.uint8)) == b"[]"


def test_base64_padding_only_at_text_end(ctx):
    """'=' in the last chars of an interior host batch is an illegal character,
    not padding (the batch is not the end of the text)."""
    raw = np.random.default_rng(9).integers(0, 256, 3 * 40_000, dtype=np.uint8).tobytes()
    enc = bytearray(base64.b64encode(raw))
    enc[16 * 4096 - 1] = ord("=")
    ctx.set_batch_words(4096)  # decode batches of 4096 16-char units
    try:
        with pytest.raises(ValueError, match="index %d" % (16 * 4096 - 1)):
            ctx.base64_decode(bytes(enc))
    finally:
        ctx.set_batch_words(4 << 20)


@pytest.mark.parametrize("devices", [None, [0, 0, 0]])
def test_base64_bad_index_in_later_batches(ctx, devices):
    """The reported index of an illegal character is a character offset into
    the whole text, whichever host batch (16 characters per batch unit) or
    device shard it falls in."""
    import amphora_amd as A
    c = ctx if devices is None else A.Context(P, R, RINV, devices=devices)
    raw = np.random.default_rng(11).integers(0, 256, 3 * 200_000, dtype=np.uint8).tobytes()
    good = base64.b64encode(raw)
    c.set_batch_words(4096)  # 65 536 characters per batch
    try:
        for where in (16 * 4096 + 5, 2 * 16 * 4096 + 16 * 100 + 7, 5 * 16 * 4096, len(good) - 9,
                      len(good) // 3 + 1, 2 * len(good) // 3 + 3):
            bad = bytearray(good)
            bad[where] = ord("*")
            with pytest.raises(ValueError, match="index %d$" % where):
                c.base64_decode(bytes(bad))
        # two bad characters: the smaller index wins across batches
        bad = bytearray(good)
        bad[3 * 16 * 4096 + 1] = ord("!")
        bad[16 * 4096 + 2] = ord("!")
        with pytest.raises(ValueError, match="index %d$" % (16 * 4096 + 2)):
            c.base64_decode(bytes(bad))
        assert c.base64_decode(good) == raw
    finally:
        c.set_batch_words(4 << 20)


@pytest.mark.parametrize("off", [0, 1, 4, 8])
def test_base64_device_alignment(ctx, off):
    """Bulk (LDS-staged) and per-lane kernels agree for aligned and
    misaligned device buffers, with a bad character in the bulk range."""
    import torch
    raw = np.random.default_rng(off).integers(0, 256, 3 * 100_003 + 2, dtype=np.uint8).tobytes()
    exp = base64.b64encode(raw)
    t = torch.zeros(len(raw) + 16, dtype=torch.uint8, device="cuda")
    t[off:off + len(raw)] = torch.frombuffer(bytearray(raw), dtype=torch.uint8).cuda()
    enc = ctx.base64_encode(t[off:off + len(raw)])
    assert enc.cpu().numpy().tobytes() == exp
    e2 = torch.zeros(len(exp) + 16, dtype=torch.uint8, device="cuda")
    e2[off:off + len(exp)] = enc
    dec, bad = ctx.base64_decode(e2[off:off + len(exp)])
    assert dec.cpu().numpy().tobytes() == raw and int(bad.item()) == 0x7F7F7F7F7F7F7F7F
    e2[off + 50_001] = ord("?")
    _, bad = ctx.base64_decode(e2[off:off + len(exp)])
    assert int(bad.item()) == 50_001


def test_vss_json_tags_named_like_fields(ctx):
    """Tags whose keys or values are the ODO member names (they come before
    the members in the document) do not shadow the members."""
    import amphora_amd as A
    from amphora_amd import wire
    odo = A.OutputDeliveryObject(b"s" * 32, b"r" * 32, b"v" * 32, b"w" * 32, b"u" * 32)
    sid = uuid.UUID("80fbba1b-3da8-4b1e-8a2c-cebd65229fad")
    tags = [{"key": "rShares", "value": "secretShares"}, {"key": "uShares", "value": 'say "wShares"'}]
    for pretty in (True, False):
        text = wire.vss_to_json(ctx, sid, tags, odo, pretty=pretty)
        sid2, tags2, odo2 = wire.vss_from_json(ctx, text)
        assert sid2 == sid and odo2 == odo
        assert [(t["key"], t["value"]) for t in tags2] == [(t["key"], t["value"]) for t in tags]


def test_vss_json_malformed_fields_are_client_errors(ctx):
    """A party body with a field that is not a whole number of words, or
    with fields of unequal length, is an AmphoraClientException;
    the secretId returned is the one requested (DefaultAmphoraClient.java:213-216)."""
    import amphora_amd as A
    from amphora_amd import client, wire
    from oracle import coracle
    F = coracle.test_field(threads=4)
    util = client.SecretShareUtil.of(P, R, RINV)
    odos, _ = F.synth_odos(seed=31, n=2, W=40)
    sid = uuid.UUID("80fbba1b-3da8-4b1e-8a2c-cebd65229fad")
    asked = uuid.UUID("00000000-0000-4000-8000-000000000001")
    names = ("secretShares", "rShares", "vShares", "wShares", "uShares")

    def bodies(cut=None):  # cut(j, k) -> bytes to drop from party j's field k
        out = []
        for j, o in enumerate(odos):
            f = [bytes(np.ascontiguousarray(x).tobytes()) for x in o]
            d = json.loads(wire.vss_to_json(ctx, sid, [], A.OutputDeliveryObject(*f), pretty=False))
            for k in range(5):
                c = cut(j, k) if cut else 0
                if c:
                    d[names[k]] = base64.b64encode(f[k][:-c]).decode()
            out.append(json.dumps(d, separators=(",", ":")))
        return out

    got_sid, _, ys = client.verify_vss_json(util, bodies(), asked)
    assert got_sid == asked
    assert ys == [int.from_bytes(w.tobytes(), "little") for w in F.recombine_verify(odos)[0]]
    with pytest.raises(A.AmphoraClientException):  # 15 bytes short of a whole word
        client.verify_vss_json(util, bodies(lambda j, k: 1 if j == 0 else 0))
    with pytest.raises(A.AmphoraClientException, match="same length"):
        client.verify_vss_json(util, bodies(lambda j, k: 16 if (j, k) == (1, 2) else 0))
    with pytest.raises(A.AmphoraClientException):  # one whole party a word short
        client.verify_vss_json(util, bodies(lambda j, k: 16 if j == 1 else 0))


@pytest.mark.parametrize("nbytes", [12 * 256, 12 * 256 + 1, 12 * 512, 12 * 512 - 2, 12 * 257, 12 * 256 * 3 + 11])
@pytest.mark.parametrize("offset", [0, 1])
def test_base64_block_kernels_tail_workgroup(ctx, nbytes, offset):
    """The block kernels take the stream's remaining units (1..256, the final
    one partial / padded) as their last workgroup: sizes at and around the
    256-unit block boundaries, 16-byte-aligned buffers (block path) and a
    1-byte offset (per-lane path), encode and decode, with the async decode
    and a bad character placed in the tail workgroup's units."""
    import torch
    raw = np.random.default_rng(nbytes + offset).integers(0, 256, nbytes, dtype=np.uint8).tobytes()
    exp = base64.b64encode(raw)
    buf = torch.zeros(nbytes + 16, dtype=torch.uint8, device="cuda")
    t = buf[offset:offset + nbytes]
    t.copy_(torch.frombuffer(bytearray(raw), dtype=torch.uint8).cuda())
    enc = ctx.base64_encode(t)
    assert enc.cpu().numpy().tobytes() == exp
    tb = torch.zeros(len(exp) + 16, dtype=torch.uint8, device="cuda")
    te = tb[offset:offset + len(exp)]
    te.copy_(enc)
    dec, bad = ctx.base64_decode(te)
    assert dec.cpu().numpy().tobytes() == raw and int(bad.item()) == 0x7F7F7F7F7F7F7F7F
    dec2, bad2 = ctx.base64_decode(te, nbytes)
    assert dec2.cpu().numpy().tobytes() == raw and int(bad2.item()) == 0x7F7F7F7F7F7F7F7F
    pos = len(exp) - 7  # inside the last units
    bt = bytearray(exp)
    bt[pos] = ord("#")
    te.copy_(torch.frombuffer(bt, dtype=torch.uint8).cuda())
    _, bad3 = ctx.base64_decode(te, nbytes)
    assert int(bad3.item()) == pos
