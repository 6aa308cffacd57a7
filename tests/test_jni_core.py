"""The JNI layer (jni/amphora_jni.c + jni/amphora_jni_core.c) driven through a
mock JNIEnv (tests/jni_mock/, test harness only -- no JDK exists here).

CPU: the status -> Java exception mapping; argument and length checks that
must fire before anything reaches the C ABI (a Java byte[] shorter than the
word count implies would otherwise be read or written past its end); the
JNI rules -- no JNI call inside a critical region, every pinned array
released, inputs released with JNI_ABORT and outputs committed.
GPU: every Java entry point against the C oracle / the ABI through Python on
the same inputs -- the client's recombineVerify / maskInput / verify /
recombine / maskWords / verifyMessage / the base64 variants, the service's
convertShare / odoPre / exchange encode+decode / openPost (a 2-party Output
Delivery run entirely through the JNI entry points).
"""
import base64
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from oracle import amphora_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MOCK = os.path.join(ROOT, "tests", "jni_mock", "libjni_mock.so")
P, R, RINV = O.TEST_PRIME, O.TEST_R, O.TEST_RINV
CLIENT = "Java_io_carbynestack_amphora_client_NativeShareArithmetic_"
SERVICE = "Java_io_carbynestack_amphora_service_calculation_NativeShareArithmetic_"
IAE = "java/lang/IllegalArgumentException"


@pytest.fixture(scope="module")
def J():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "jni"), "mock"], check=True)
    # amphora_amd first: it loads torch's HIP runtime before libamphora_hip, so
    # the mock's libamphora_hip binds to that one instance (a process whose first
    # HIP library is /opt/rocm's sees no device through torch's, and vice versa)
    import amphora_amd  # noqa: F401
    L = C.CDLL(MOCK)
    vp = C.c_void_p
    L.mock_env.restype = vp
    for f in ("mock_bytes", "mock_ints", "mock_objects"):
        getattr(L, f).restype = vp
    L.mock_bytes.argtypes = [C.c_char_p, C.c_int32]
    L.mock_ints.argtypes = [C.POINTER(C.c_int32), C.c_int32]
    L.mock_objects.argtypes = [C.POINTER(vp), C.c_int32]
    L.mock_len.argtypes = [vp]
    L.mock_data.restype = vp
    L.mock_data.argtypes = [vp]
    L.mock_commits.argtypes = L.mock_aborts.argtypes = [vp]
    L.mock_region_copies.restype = C.c_long
    L.mock_exception_class.restype = L.mock_exception_message.restype = C.c_char_p
    L.amphj_exception_class.restype = C.c_char_p
    return L


class Env:
    """Java-side helpers over the mock: arrays in, results out."""

    def __init__(self, L):
        self.L = L
        self.env = L.mock_env()
        L.mock_free_all()

    def bytes(self, b):
        b = bytes(np.ascontiguousarray(b).tobytes()) if isinstance(b, np.ndarray) else bytes(b)
        return self.L.mock_bytes(b, len(b))

    def zeros(self, n):
        return self.L.mock_bytes(None, n)

    def objects(self, objs):
        arr = (C.c_void_p * len(objs))(*objs)
        return self.L.mock_objects(arr, len(objs))

    def read(self, obj):
        n = self.L.mock_len(obj)
        return C.string_at(self.L.mock_data(obj), n) if n > 0 else b""

    def call(self, name, restype, *args):
        fn = getattr(self.L, name)
        fn.restype = restype
        conv = [C.c_void_p(self.env), C.c_void_p(None)]
        for a in args:
            conv.append(a if isinstance(a, C._SimpleCData) else C.c_void_p(a))
        return fn(*conv)

    def exception(self):
        cls = self.L.mock_exception_class().decode()
        return (cls, self.L.mock_exception_message().decode()) if cls else None

    def clean(self):
        """JNI rules held: nothing called inside a critical region, nothing left pinned."""
        return self.L.mock_violations() == 0 and self.L.mock_open_criticals() == 0

    def odo_lists(self, odos):
        return [self.objects([self.bytes(o[k]) for o in odos]) for k in range(5)]


def le16(x):
    return int(x).to_bytes(16, "little")


def test_exception_mapping(J):
    assert J.amphj_exception_class(0) is None
    assert J.amphj_exception_class(1) == b"io/carbynestack/amphora/common/exceptions/IntegrityVerificationException"
    assert J.amphj_exception_class(2) == J.amphj_exception_class(3) == IAE.encode()
    assert J.amphj_exception_class(4) == J.amphj_exception_class(5) == b"java/lang/IllegalStateException"
    assert J.amphj_exception_class(6) == b"java/lang/ArrayIndexOutOfBoundsException"


def test_checks_fire_before_the_abi(J):
    """No context is needed: each case is rejected before libamphora_hip is called."""
    e = Env(J)
    ctx = C.c_int64(0)
    word = e.bytes(b"\0" * 32)
    short = e.bytes(b"\0" * 16)
    # parties out of range
    empty = e.objects([])
    assert e.call(CLIENT + "recombineVerify", C.c_int64, ctx, empty, empty, empty, empty, empty, e.zeros(32)) == -1
    assert e.exception() == (IAE, "n_parties must be in [1, 16]") and e.clean()
    # one field shorter than the others (ADVICE r2's over-read, at the JNI boundary)
    J.mock_clear()
    lists = [e.objects([word, word]) for _ in range(4)] + [e.objects([word, short])]
    assert e.call(CLIENT + "recombineVerify", C.c_int64, ctx, *lists, e.zeros(32)) == -1
    assert e.exception() == (IAE, "The provided shares must be of the same length") and e.clean()
    # output array too short for the words
    J.mock_clear()
    lists = [e.objects([word, word]) for _ in range(5)]
    out = e.zeros(16)
    e.call(CLIENT + "recombineVerify", C.c_int64, ctx, *lists, out)
    cls, msg = e.exception()
    assert cls == IAE and "secrets array holds 16 bytes, 32 needed" in msg and e.clean()
    assert J.mock_aborts(word) >= 1 and J.mock_commits(word) == 0  # inputs never copied back
    assert J.mock_commits(out) == 1
    # service: SecretShareUtil.java:64-66
    J.mock_clear()
    e.call(SERVICE + "convertShare", None, ctx, e.bytes(b"\0" * 32), e.bytes(b"\0" * 32), e.bytes(b"\0" * 16),
           C.c_uint8(0), e.zeros(64))
    assert e.exception() == (IAE, "Received more input data than available inputMasks.") and e.clean()
    # odoPre: the triple stream must hold 2W triples
    J.mock_clear()
    e.call(SERVICE + "odoPre", None, ctx, e.bytes(b"\0" * 64), C.c_int32(32), e.bytes(b"\0" * 128),
           e.bytes(b"\0" * 100), e.zeros(32), e.zeros(32), e.zeros(32), e.zeros(128), e.zeros(8))
    cls, msg = e.exception()
    assert cls == IAE and "triple stream" in msg and e.clean()
    # exchange decode span outside the body
    J.mock_clear()
    e.call(SERVICE + "exchangeDecode", None, ctx, e.bytes(b"[]"), C.c_int32(1), C.c_int32(5), C.c_int64(0),
           e.zeros(0), e.zeros(0))
    assert e.exception() == (IAE, "interimValues span outside the body") and e.clean()
    # context parameters must be 16-byte integers
    J.mock_clear()
    assert e.call(CLIENT + "ctxCreate", C.c_int64, e.bytes(b"\1" * 8), e.bytes(b"\0" * 16), e.bytes(b"\0" * 16),
                  None) == 0
    assert e.exception()[0] == IAE and e.clean()


def test_local_references_and_refused_pins(J):
    """16 parties hold 5 x 16 element references at once: the layer reserves
    them (EnsureLocalCapacity) instead of relying on the 16 a native method is
    guaranteed; a pin the VM refuses releases the pins already taken, unwritten,
    and leaves its OutOfMemoryError pending -- nothing reaches the C ABI."""
    e = Env(J)
    ctx = C.c_int64(0)
    word = e.bytes(b"\0" * 32)
    J.mock_clear()
    lists = [e.objects([word] * 16) for _ in range(5)]
    e.call(CLIENT + "recombineVerify", C.c_int64, ctx, *lists, e.zeros(16))
    cls, msg = e.exception()
    assert cls == IAE and "32 needed" in msg and e.clean()
    assert J.mock_ref_overflows() == 0
    for k in (1, 3, 11):  # the first, a middle and the output (5 x 2 fields + out) pin refused
        J.mock_clear()
        lists = [e.objects([word, word]) for _ in range(5)]
        out = e.zeros(32)
        J.mock_fail_pin(k)
        assert e.call(CLIENT + "recombineVerify", C.c_int64, ctx, *lists, out) == -1
        assert e.exception() == ("java/lang/OutOfMemoryError", "mock: pin refused") and e.clean()
        assert J.mock_commits(out) == 0 and J.mock_ref_overflows() == 0


# ---------------------------------------------------------------- GPU --------
@pytest.fixture(scope="module")
def jctx(J):
    import torch
    assert torch.cuda.is_available()
    e = Env(J)
    h = e.call(CLIENT + "ctxCreate", C.c_int64, e.bytes(le16(P)), e.bytes(le16(R)), e.bytes(le16(RINV)), None)
    assert h != 0 and e.exception() is None
    yield h
    Env(J).call(CLIENT + "ctxDestroy", None, C.c_int64(h))


@pytest.fixture(scope="module")
def F():
    from oracle import coracle
    return coracle.test_field(threads=8)


@pytest.mark.gpu
@pytest.mark.parametrize("n,W", [(2, 1000), (3, 5000), (2, 70_000)])
def test_client_entry_points(J, jctx, F, n, W):
    e = Env(J)
    ctx = C.c_int64(jctx)
    odos, _ = F.synth_odos(seed=W + n, n=n, W=W, noncanon_permille=10)
    oy, off = F.recombine_verify(odos)
    out = e.zeros(16 * W)
    assert e.call(CLIENT + "recombineVerify", C.c_int64, ctx, *e.odo_lists(odos), out) == -1
    assert e.exception() is None and e.clean() and e.read(out) == oy.tobytes()
    bad, _ = F.synth_odos(seed=W + n, n=n, W=W, fault_index=W // 3)
    assert e.call(CLIENT + "recombineVerify", C.c_int64, ctx, *e.odo_lists(bad), e.zeros(16 * W)) == W // 3
    assert e.exception() is None  # a verify failure is returned, the Java side renders the message
    secrets = F.synth_words(seed=7, count=W - 3, mont=False)
    om, _ = F.mask_input(secrets, [tuple(f[: W - 3] for f in o) for o in odos])
    out = e.zeros(16 * (W - 3))
    assert e.call(CLIENT + "maskInput", C.c_int64, ctx, *e.odo_lists(odos), e.bytes(secrets), out) == -1
    assert e.read(out) == om.tobytes() and e.clean()
    # recombine / verify / maskWords on the recombined fields
    f = [F.recombine([o[k] for o in odos]) for k in range(5)]  # y, r, v, w, u canonical
    out = e.zeros(16 * W)
    e.call(CLIENT + "recombine", None, ctx, e.objects([e.bytes(o[0]) for o in odos]), out)
    assert e.read(out) == f[0].tobytes()
    assert e.call(CLIENT + "verify", C.c_int64, ctx, *[e.bytes(f[k]) for k in (0, 1, 4, 2, 3)]) == -1
    f3 = f[3].copy()
    f3[W // 2, 0] ^= 1
    assert e.call(CLIENT + "verify", C.c_int64, ctx, e.bytes(f[0]), e.bytes(f[1]), e.bytes(f[4]), e.bytes(f[2]),
                  e.bytes(f3)) == W // 2
    masks = F.synth_words(seed=8, count=W, mont=False)
    out = e.zeros(16 * W)
    e.call(CLIENT + "maskWords", None, ctx, e.bytes(secrets[:W // 2]), e.bytes(masks[:W // 2]), out)
    exp = b"".join(((((int.from_bytes(s.tobytes(), "little") - int.from_bytes(m.tobytes(), "little")) % P) * R % P)
                    .to_bytes(16, "little")) for s, m in zip(secrets[:W // 2], masks[:W // 2]))
    assert e.read(out)[: len(exp)] == exp and e.clean()


@pytest.mark.gpu
def test_client_text_entry_points_and_message(J, jctx, F):
    import amphora_amd as A
    e = Env(J)
    ctx = C.c_int64(jctx)
    W, n = 3000, 2
    odos, _ = F.synth_odos(seed=5, n=n, W=W)
    texts = [[base64.b64encode(np.ascontiguousarray(f).tobytes()) for f in o] for o in odos]
    tl = [e.objects([e.bytes(t[k]) for t in texts]) for k in range(5)]
    out = e.zeros(16 * W)
    assert e.call(CLIENT + "recombineVerifyB64", C.c_int64, ctx, *tl, C.c_int64(W), out) == -1
    assert e.read(out) == F.recombine_verify(odos)[0].tobytes() and e.clean()
    secrets = F.synth_words(seed=6, count=W, mont=False)
    rec = e.zeros(24 * W)
    assert e.call(CLIENT + "maskInputB64", C.c_int64, ctx, *tl, C.c_int64(W), e.bytes(secrets), rec) == -1
    om, _ = F.mask_input(secrets, odos)
    assert e.read(rec) == b"".join(base64.b64encode(w.tobytes()) for w in om)
    # a bad character: IllegalArgumentException naming party, field, offset
    t2 = bytearray(texts[1][2])
    t2[77] = ord("*")
    tl[2] = e.objects([e.bytes(texts[0][2]), e.bytes(bytes(t2))])
    J.mock_clear()
    e.call(CLIENT + "recombineVerifyB64", C.c_int64, ctx, *tl, C.c_int64(W), e.zeros(16 * W))
    cls, msg = e.exception()
    assert cls == IAE and "index 77 of party 1's vShares" in msg and e.clean()
    # the reference's failure text (SecretShareUtil.java:116-129)
    ref = A.Context(P, R, RINV)
    vals = [12345, 678, 91011, 1213, 1415]
    s = e.call(CLIENT + "verifyMessage", C.c_void_p, ctx, *[e.bytes(le16(x)) for x in vals])
    assert e.read(s).decode() == ref.verify_message(*vals)


@pytest.mark.gpu
def test_service_entry_points_two_party_output_delivery(J, jctx, F):
    """convertShare (KAT-free, against the oracle) and a full 2-party Output
    Delivery through odoPre -> exchangeEncode -> exchangeDecode -> openPost."""
    e = Env(J)
    ctx = C.c_int64(jctx)
    W = 777
    masked = F.synth_words(seed=11, count=W)
    tuples = F.synth_words(seed=12, count=2 * W).reshape(W, 32)
    key = 0x1234567890ABCDEF1234567890ABCD % P
    for use_zero in (0, 1):
        out = e.zeros(32 * W)
        e.call(SERVICE + "convertShare", None, ctx, e.bytes(masked), e.bytes(tuples), e.bytes(le16(key)),
               C.c_uint8(use_zero), out)
        assert e.exception() is None and e.clean()
        assert e.read(out) == F.convert_share(masked, tuples, key, bool(use_zero)).tobytes()
    # Output Delivery: each party's share data (stride 32), masks (2W x 32 B), triples (2W x 96 B)
    shares = [F.synth_words(seed=20 + j, count=2 * W).reshape(W, 32) for j in range(2)]
    masks = [F.synth_words(seed=30 + j, count=4 * W).reshape(2 * W, 32) for j in range(2)]
    triples = [F.synth_words(seed=40 + j, count=12 * W).reshape(2 * W, 96) for j in range(2)]
    pre, texts = [], []
    for j in range(2):
        y, r, v, mag, neg = (e.zeros(16 * W), e.zeros(16 * W), e.zeros(16 * W), e.zeros(64 * W), e.zeros(4 * W))
        e.call(SERVICE + "odoPre", None, ctx, e.bytes(shares[j]), C.c_int32(32), e.bytes(masks[j]),
               e.bytes(triples[j]), y, r, v, mag, neg)
        assert e.exception() is None and e.clean()
        oy, orr, ov, omag, oneg = F.odo_pre(shares[j], 32, masks[j], triples[j])
        assert [e.read(x) for x in (y, r, v, mag, neg)] == [a.tobytes() for a in (oy, orr, ov, omag, oneg)]
        txt = e.call(SERVICE + "exchangeEncode", C.c_void_p, ctx, mag, neg)
        assert e.exception() is None and e.read(txt).startswith(b'[{"a":')
        pre.append((omag, oneg))
        texts.append(e.read(txt))
    for j in range(2):
        mags, negs = [], []
        for k in (j, 1 - j):  # own diffs first, then the partner's decoded from its text
            body = b'{"interimValues":' + texts[k] + b"}"
            mag, neg = e.zeros(64 * W), e.zeros(4 * W)
            e.call(SERVICE + "exchangeDecode", None, ctx, e.bytes(body), C.c_int32(17), C.c_int32(len(texts[k])),
                   C.c_int64(2 * W), mag, neg)
            assert e.exception() is None and e.clean()
            assert e.read(mag) == pre[k][0].tobytes() and e.read(neg) == pre[k][1].tobytes()
            mags.append(mag)
            negs.append(neg)
        w, u = e.zeros(16 * W), e.zeros(16 * W)
        e.call(SERVICE + "openPost", None, ctx, e.objects(mags), e.objects(negs), e.bytes(triples[j]),
               C.c_uint8(j == 0), w, u)
        assert e.exception() is None and e.clean()
        opened = F.recombine_diffs([pre[j][0], pre[1 - j][0]], [pre[j][1], pre[1 - j][1]])
        ow, ou = F.odo_post(opened, triples[j], j == 0)
        assert e.read(w) == ow.tobytes() and e.read(u) == ou.tobytes()


def test_party_session_checks_before_the_abi(J):
    """Session entry points: argument and length checks before libamphora_hip."""
    e = Env(J)
    ctx = C.c_int64(0)
    W = 10
    share, masks, triples = e.bytes(b"\0" * 32 * W), e.bytes(b"\0" * 64 * W), e.bytes(b"\0" * 192 * W)
    J.mock_clear()
    assert e.call(SERVICE + "partyBegin", C.c_int64, ctx, share, C.c_int32(24), masks, triples, C.c_int32(2),
                  None, None, None) == 0
    assert e.exception() == (IAE, "share stride must be 16 or 32") and e.clean()
    J.mock_clear()
    e.call(SERVICE + "partyBegin", C.c_int64, ctx, share, C.c_int32(32), e.bytes(b"\0" * 64 * W),
           e.bytes(b"\0" * 100), C.c_int32(2), None, None, None)
    cls, msg = e.exception()
    assert cls == IAE and "triple stream" in msg and e.clean()
    J.mock_clear()  # y/r/v all or none
    e.call(SERVICE + "partyBegin", C.c_int64, ctx, share, C.c_int32(32), masks, triples, C.c_int32(2),
           e.zeros(16 * W), None, None)
    assert e.exception()[0] == IAE and e.clean()
    J.mock_clear()
    e.call(SERVICE + "partyPartner", None, C.c_int64(0), C.c_int32(1), e.bytes(b"[]"), C.c_int32(0), C.c_int32(5))
    assert e.exception() == (IAE, "interimValues span outside the body") and e.clean()
    J.mock_clear()
    e.call(SERVICE + "partyText", C.c_void_p, C.c_int64(0))
    assert e.exception() == (IAE, "null party session") and e.clean()
    J.mock_clear()
    e.call(SERVICE + "partyFinishBase64", None, C.c_int64(0), C.c_uint8(1), e.objects([e.zeros(4)] * 4))
    assert e.exception()[0] == IAE and e.clean()


@pytest.mark.gpu
def test_service_party_session_three_parties(J, jctx, F):
    """A 3-party Output Delivery through the session entry points (partyBegin ->
    partyText -> partyPartner x 2 -> partyFinish / partyFinishBase64) against
    the oracle; inputs pinned with JNI_ABORT, outputs committed."""
    e = Env(J)
    ctx = C.c_int64(jctx)
    n, W = 3, 1234
    shares = [F.synth_words(seed=50 + j, count=2 * W).reshape(W, 32) for j in range(n)]
    masks = [F.synth_words(seed=60 + j, count=4 * W).reshape(2 * W, 32) for j in range(n)]
    triples = [F.synth_words(seed=70 + j, count=12 * W).reshape(2 * W, 96) for j in range(n)]
    pre = [F.odo_pre(shares[j], 32, masks[j], triples[j]) for j in range(n)]
    handles, texts, yrv = [], [], []
    for j in range(n):
        fields = (e.zeros(16 * W), e.zeros(16 * W), e.zeros(16 * W)) if j < 2 else (None, None, None)
        share_arr = e.bytes(shares[j])
        h = e.call(SERVICE + "partyBegin", C.c_int64, ctx, share_arr, C.c_int32(32), e.bytes(masks[j]),
                   e.bytes(triples[j]), C.c_int32(n), *fields)
        assert h != 0 and e.exception() is None and e.clean()
        if os.environ.get("AMPH_JNI_REGION_BYTES") != "0":  # pinned: inputs released unwritten
            assert J.mock_aborts(share_arr) == 1 and J.mock_commits(share_arr) == 0
        if j < 2:
            assert [e.read(x) for x in fields] == [pre[j][k].tobytes() for k in range(3)]
        txt = e.call(SERVICE + "partyText", C.c_void_p, C.c_int64(h))
        assert e.exception() is None and e.clean()
        handles.append(h)
        texts.append(e.read(txt))
        yrv.append(fields)
    for j in range(n):
        h = C.c_int64(handles[j])
        for slot, k in enumerate([k for k in range(n) if k != j], start=1):
            body = b'{"operationId":"x","playerId":%d,"interimValues":' % k + texts[k] + b"}"
            off = body.index(b"[")
            e.call(SERVICE + "partyPartner", None, h, C.c_int32(slot), e.bytes(body), C.c_int32(off),
                   C.c_int32(len(texts[k])))
            assert e.exception() is None and e.clean()
        opened = F.recombine_diffs([pre[k][3] for k in range(n)], [pre[k][4] for k in range(n)])
        ow, ou = F.odo_post(opened, triples[j], j == 0)
        if j < 2:
            w, u = e.zeros(16 * W), e.zeros(16 * W)
            e.call(SERVICE + "partyFinish", None, h, C.c_uint8(j == 0), w, u)
            assert e.exception() is None and e.clean()
            assert e.read(w) == ow.tobytes() and e.read(u) == ou.tobytes()
        else:
            nc = 4 * ((16 * W + 2) // 3)
            outs = [e.zeros(nc) for _ in range(5)]
            e.call(SERVICE + "partyFinishBase64", None, h, C.c_uint8(0), e.objects(outs))
            assert e.exception() is None and e.clean()
            want = [base64.b64encode(x.tobytes()) for x in (pre[j][0], pre[j][1], pre[j][2], ow, ou)]
            assert [e.read(o) for o in outs] == want
        # a second finish is an error (the session is spent)
        J.mock_clear()
        e.call(SERVICE + "partyFinish", None, h, C.c_uint8(0), e.zeros(16 * W), e.zeros(16 * W))
        assert e.exception() == (IAE, "the party session is already finished") and e.clean()
        J.mock_clear()
        e.call(SERVICE + "partyFree", None, h)


def test_mask_word_makes_no_launch(J):
    """the per-word maskInput (SecretShareUtil.java:65-68,
    called once per word from DefaultAmphoraClient.java:155-160's parallel
    stream) goes through maskWord: two 16-byte region copies in, host
    arithmetic, one array out -- no critical region, no kernel launch (the
    context's launch counter stays 0), and toGfp((s - m) mod p) exactly.
    Needs no GPU: nothing here touches the device."""
    import random
    import amphora_amd as A
    e = Env(J)
    h = e.call(CLIENT + "ctxCreate", C.c_int64, e.bytes(le16(P)), e.bytes(le16(R)), e.bytes(le16(RINV)), None)
    assert h != 0 and e.exception() is None
    rnd = random.Random(11)
    cases = [(0, 0), (5, 7), (P - 1, 1), (1, P - 1), (P - 1, P - 1)] + \
            [(rnd.randrange(P), rnd.randrange(P)) for _ in range(200)]
    for s, m in cases:
        J.mock_clear()
        out = e.call(CLIENT + "maskWord", C.c_void_p, C.c_int64(h), e.bytes(le16(s)), e.bytes(le16(m)))
        assert e.exception() is None and e.clean()
        assert e.read(out) == le16((s - m) % P * R % P), (s, m)
        assert J.mock_pins() == 0  # region copies only
    stats = A._lib._AmphStats()
    assert A._lib.lib.amph_ctx_stats(C.c_void_p(h), C.byref(stats)) == 0
    assert stats.kernel_launches == 0
    # wrong word sizes are refused before the ABI
    J.mock_clear()
    assert e.call(CLIENT + "maskWord", C.c_void_p, C.c_int64(h), e.bytes(b"\1" * 8), e.bytes(le16(1))) is None
    assert e.exception() == (IAE, "maskWord takes two 16-byte words") and e.clean()
    Env(J).call(CLIENT + "ctxDestroy", None, C.c_int64(h))


# ---- large calls: region copies, no critical region across the GPU call -------
@pytest.mark.gpu
@pytest.mark.parametrize("n,W", [(2, 70_000), (3, 300_000)])
def test_client_entry_points_region_mode(J, jctx, F, n, W, monkeypatch):
    """above AMPH_JNI_REGION_BYTES (forced to 0 here) the
    client entry points pin nothing: libamphora_hip's staging threads move
    each batch with Get/SetByteArrayRegion (AMPH_F_HOST_IO), attached to the
    VM as daemons; every result still equals the oracle's, and every global
    reference is released."""
    monkeypatch.setenv("AMPH_JNI_REGION_BYTES", "0")
    J.mock_clear()
    test_client_entry_points(J, jctx, F, n, W)
    assert J.mock_pins() == 0, "a critical region was opened above the threshold"
    assert J.mock_region_copies() > 0 and J.mock_global_refs() == 0
    if 16 * W * (5 * n + 1) > (2 << 20):  # the batched pipeline: copies on the staging threads
        assert J.mock_foreign_regions() > 0 and J.mock_attaches() > 0
    assert J.mock_violations() == 0 and J.mock_open_criticals() == 0


@pytest.mark.gpu
def test_service_entry_points_region_mode(J, jctx, F, monkeypatch):
    monkeypatch.setenv("AMPH_JNI_REGION_BYTES", "0")
    J.mock_clear()
    test_service_entry_points_two_party_output_delivery(J, jctx, F)
    # exchangeEncode / exchangeDecode keep their (short, text-sized) pins; the
    # word-array calls convertShare / odoPre / openPost took none
    assert J.mock_global_refs() == 0 and J.mock_violations() == 0 and J.mock_open_criticals() == 0
    assert J.mock_region_copies() > 0


@pytest.mark.gpu
def test_party_session_region_mode(J, jctx, F, monkeypatch):
    """above the threshold the session calls copy their arrays
    into native buffers with region copies -- nothing stays pinned while a
    session call waits for the context or the GPU."""
    monkeypatch.setenv("AMPH_JNI_REGION_BYTES", "0")
    J.mock_clear()
    test_service_party_session_three_parties(J, jctx, F)
    assert J.mock_pins() == 0 and J.mock_open_criticals() == 0 and J.mock_violations() == 0


@pytest.mark.gpu
def test_small_calls_still_pin(J, jctx, F, monkeypatch):
    """Below the default threshold (2 MiB of arrays) a call pins: short
    critical regions are cheaper than region copies."""
    monkeypatch.delenv("AMPH_JNI_REGION_BYTES", raising=False)
    J.mock_clear()
    e = Env(J)
    odos, _ = F.synth_odos(seed=3, n=2, W=1000)
    out = e.zeros(16 * 1000)
    assert e.call(CLIENT + "recombineVerify", C.c_int64, C.c_int64(jctx), *e.odo_lists(odos), out) == -1
    assert e.read(out) == F.recombine_verify(odos)[0].tobytes()
    assert J.mock_pins() == 11 and J.mock_region_copies() == 0 and e.clean()


# ---- recombineObject's ragged party arrays through JNI (SecretShareUtil.java:70-90)
AIOOBE = "java/lang/ArrayIndexOutOfBoundsException"


@pytest.mark.gpu
@pytest.mark.parametrize("region", [False, True])
@pytest.mark.parametrize("delta,outcome", [(53, "ok"), (-8, "pad"), (-32, "range")])
def test_client_ragged_partner(J, jctx, F, delta, outcome, region, monkeypatch):
    """A partner whose ODO arrays are longer (cut), short by 8 bytes (last
    word zero-padded: MAC failure at W-1, the padded word recombined) or
    short by two words (ArrayIndexOutOfBoundsException), through
    recombineVerify, maskInput and recombine, pinned and region-copied --
    each against the oracle's restatement of copyOfRange."""
    from tests.test_ragged_parties import _ragged
    from oracle import amphora_oracle as O
    if region:
        monkeypatch.setenv("AMPH_JNI_REGION_BYTES", "0")
    else:
        monkeypatch.delenv("AMPH_JNI_REGION_BYTES", raising=False)
    e = Env(J)
    ctx = C.c_int64(jctx)
    W, n = 5000, 3
    odos = _ragged(F, W, n, delta, seed=71)
    secrets = F.synth_words(seed=72, count=W, mont=False)
    J.mock_clear()
    out = e.zeros(16 * W)
    got = e.call(CLIENT + "recombineVerify", C.c_int64, ctx, *e.odo_lists(odos), out)
    if outcome == "range":
        assert got == -1 and e.exception()[0] == AIOOBE and e.clean()
        with pytest.raises(O.ArrayIndexOutOfBoundsException):
            F.recombine_verify_object(odos)
        J.mock_clear()
        e.call(CLIENT + "maskInput", C.c_int64, ctx, *e.odo_lists(odos), e.bytes(secrets), e.zeros(16 * W))
        assert e.exception()[0] == AIOOBE and e.clean()
        J.mock_clear()
        e.call(CLIENT + "recombine", None, ctx, e.objects([e.bytes(o[0]) for o in odos]), e.zeros(16 * W))
        assert e.exception()[0] == AIOOBE and e.clean()
        return
    ey, eff = F.recombine_verify_object(odos)
    assert got == eff == (-1 if outcome == "ok" else W - 1)
    assert e.exception() is None and e.clean() and e.read(out) == ey.tobytes()
    out = e.zeros(16 * W)
    em, mff = F.mask_input_object(secrets, odos)
    assert e.call(CLIENT + "maskInput", C.c_int64, ctx, *e.odo_lists(odos), e.bytes(secrets), out) == mff
    assert e.exception() is None and e.clean() and e.read(out) == em.tobytes()
    out = e.zeros(16 * W)
    e.call(CLIENT + "recombine", None, ctx, e.objects([e.bytes(o[4]) for o in odos]), out)
    assert e.exception() is None and e.read(out) == F.recombine_object([o[4] for o in odos]).tobytes()
    if region:
        assert J.mock_pins() == 0


@pytest.mark.gpu
def test_staging_threads_detach_when_the_context_goes(J, F, monkeypatch):
    """libamphora_hip's staging threads attach to the VM as daemons
    for the region-copy callbacks; each must detach before it exits (JNI
    spec).  A context of its own, large calls in region mode, then
    ctxDestroy (which joins the threads): every attach is matched by a
    detach, and the calling Java thread is never detached."""
    monkeypatch.setenv("AMPH_JNI_REGION_BYTES", "0")
    J.mock_detaches.restype = J.mock_bad_detaches.restype = C.c_int
    a0, d0 = J.mock_attaches(), J.mock_detaches()
    e = Env(J)
    h = e.call(CLIENT + "ctxCreate", C.c_int64, e.bytes(le16(P)), e.bytes(le16(R)), e.bytes(le16(RINV)), None)
    assert h != 0 and e.exception() is None
    W, n = 300_000, 3
    odos, _ = F.synth_odos(seed=91, n=n, W=W)
    out = e.zeros(16 * W)
    assert e.call(CLIENT + "recombineVerify", C.c_int64, C.c_int64(h), *e.odo_lists(odos), out) == -1
    assert e.read(out) == F.recombine_verify(odos)[0].tobytes()
    attached = J.mock_attaches() - a0
    assert attached > 0, "the batched pipeline's staging threads ran the callbacks"
    Env(J).call(CLIENT + "ctxDestroy", None, C.c_int64(h))
    assert J.mock_detaches() - d0 == attached
    assert J.mock_bad_detaches() == 0
