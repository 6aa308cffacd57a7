"""recombineObject's ragged party arrays (client SecretShareUtil.java:70-90).

The reference takes the word count from party 0 (`shares.get(0).length /
WORD_WIDTH`, :75) and cuts every party's word i with `Arrays.copyOfRange(
share, 16 i, 16 i + 16)` (:87-88).  So a partner whose arrays are
  * longer  -> cut to party 0's word count (the extra words are never read);
  * shorter, ending inside the last word (16 (W-1) <= len < 16 W) -> that
    word zero-padded (a MAC failure at W-1 in practice, with the padded
    word's recombined value in the output);
  * shorter, ending before 16 (W-1) -> a word starts past its end:
    ArrayIndexOutOfBoundsException.
The oracles restate this (amphora_oracle.copy_of_range / recombine_object,
coracle.java_words); the C ABI (amph_recombine_verify, amph_mask_input,
amph_recombine_object: include/amphora.h `amph_odo`) matches it in host and
device mode, with AMPH_E_RANGE for the exception.  CPU tests pin the two
oracles to each other and to Java's copyOfRange; GPU tests compare the HIP
path with the C oracle bit for bit (outputs and first-fail index).
"""
import numpy as np
import pytest

from oracle import amphora_oracle as O
from oracle import coracle

P, R, RINV = O.TEST_PRIME, O.TEST_R, O.TEST_RINV
NO_FAIL = 0x7F7F7F7F7F7F7F7F

# (name, byte delta of party 1's arrays vs 16 W, expected outcome)
CASES = [("longer", 3 * 16 + 5, "ok"), ("equal", 0, "ok"), ("short8", -8, "pad"),
         ("short1", -1, "pad"), ("short16", -16, "pad"), ("short17", -17, "range"),
         ("short32", -32, "range"), ("empty", None, "range")]


def _ragged(F, W, n, delta, seed=5):
    """Honest n-party ODOs of W words; party 1's five arrays re-cut to
    16 W + delta bytes (extra bytes random), party 0's given 5 trailing bytes
    (a partial word the word count ignores)."""
    odos, _ = F.synth_odos(seed=seed, n=n, W=W)
    rng = np.random.default_rng(seed)
    out = []
    for j, o in enumerate(odos):
        fields = []
        for f in o:
            b = np.ascontiguousarray(f).reshape(-1)
            if j == 0:
                b = np.concatenate([b, rng.integers(0, 256, 5, dtype=np.uint8)])
            elif j == 1:
                if delta is None:
                    b = b[:0]
                elif delta >= 0:
                    b = np.concatenate([b, rng.integers(0, 256, delta, dtype=np.uint8)])
                else:
                    b = b[:max(0, 16 * W + delta)]
            fields.append(np.ascontiguousarray(b))
        out.append(tuple(fields))
    return out


# ---------------------------------------------------------------- CPU (oracle)
def test_copy_of_range_is_javas():
    a = bytes([1, 2, 3])
    assert O.copy_of_range(a, 0, 3) == a
    assert O.copy_of_range(a, 2, 6) == bytes([3, 0, 0, 0])
    assert O.copy_of_range(a, 3, 5) == bytes(2)  # from == length: allowed, all zeros
    with pytest.raises(O.ArrayIndexOutOfBoundsException):
        O.copy_of_range(a, 4, 6)
    with pytest.raises(O.IllegalArgumentException):
        O.copy_of_range(a, 2, 1)


@pytest.mark.parametrize("name,delta,outcome", CASES)
def test_oracles_agree_on_ragged_parties(name, delta, outcome):
    F = coracle.test_field(threads=2)
    W, n = 9, 3
    odos = _ragged(F, W, n, delta)
    util = O.ClientSecretShareUtil(P, R, RINV)
    pyodos = [O.OutputDeliveryObject(*[f.tobytes() for f in o]) for o in odos]
    if outcome == "range":
        with pytest.raises(O.ArrayIndexOutOfBoundsException):
            O.verify_output_delivery_objects(util, pyodos)
        with pytest.raises(O.ArrayIndexOutOfBoundsException):
            F.recombine_verify_object(odos)
        with pytest.raises(O.ArrayIndexOutOfBoundsException):
            F.recombine_object([o[0] for o in odos])
        return
    ys, ff = F.recombine_verify_object(odos)
    fields = [util.recombine_object([getattr(o, k) for o in pyodos]) for k in O.OutputDeliveryObject.FIELDS]
    y, r, v, w, u = fields
    assert [int.from_bytes(ys[i].tobytes(), "little") for i in range(W)] == y
    assert ff == O.first_failing_index(P, y, r, u, v, w)
    assert ff == (-1 if outcome == "ok" else W - 1)
    one = F.recombine_object([o[2] for o in odos])
    assert [int.from_bytes(one[i].tobytes(), "little") for i in range(W)] == v


# ---------------------------------------------------------------- GPU (HIP)
@pytest.fixture(scope="module")
def gpu():
    import torch
    import amphora_amd as A
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return torch, A, A.Context(P, R, RINV, device=0), coracle.test_field(threads=16)


def _on(torch, mode, odos):
    if mode == "host":
        return odos
    return [tuple(torch.from_numpy(f).cuda() for f in o) for o in odos]


def _ff(torch, ff):
    if isinstance(ff, int):
        return ff
    torch.cuda.synchronize()
    v = int(ff.cpu().item())
    return -1 if v == NO_FAIL else v


@pytest.mark.gpu
@pytest.mark.parametrize("W,n", [(4099, 2), (37, 3), (1, 2)])
@pytest.mark.parametrize("mode", ["host", "device"])
@pytest.mark.parametrize("name,delta,outcome", CASES)
def test_hip_recombine_verify_ragged(gpu, W, n, mode, name, delta, outcome):
    torch, A, ctx, F = gpu
    odos = _ragged(F, W, n, delta, seed=W + n)
    args = _on(torch, mode, odos)
    if outcome == "range" and W > 1:
        with pytest.raises(A.AmphoraNativeError) as e:
            ctx.recombine_verify(args)
        assert e.value.status == A._lib.AMPH_E_RANGE
        with pytest.raises(O.ArrayIndexOutOfBoundsException):
            F.recombine_verify_object(odos)
        return
    exp, eff = F.recombine_verify_object(odos)
    got, ff = ctx.recombine_verify(args)
    got = got if mode == "host" else got.cpu().numpy()
    assert _ff(torch, ff) == eff
    assert np.array_equal(got, exp)
    if outcome == "pad" or (outcome == "range" and W == 1):
        # W == 1: a partner of 0 bytes still reaches word 0 (copyOfRange(0, 16) of
        # an empty array is allowed): a padded word, not an exception
        assert eff == W - 1


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["host", "device"])
@pytest.mark.parametrize("secrets_short", [0, 3])
@pytest.mark.parametrize("name,delta,outcome", CASES)
def test_hip_mask_input_ragged(gpu, mode, secrets_short, name, delta, outcome):
    torch, A, ctx, F = gpu
    W, n = 2053, 3
    odos = _ragged(F, W, n, delta, seed=17)
    S = W - secrets_short
    secrets = F.synth_words(seed=18, count=S, mont=False)
    args = _on(torch, mode, odos)
    sec = secrets if mode == "host" else torch.from_numpy(secrets).cuda()
    if outcome == "range":
        with pytest.raises(A.AmphoraNativeError) as e:
            ctx.mask_input(args, sec)
        assert e.value.status == A._lib.AMPH_E_RANGE
        return
    exp, eff = F.mask_input_object(secrets, odos)
    got, ff = ctx.mask_input(args, sec)
    got = got if mode == "host" else got.cpu().numpy()
    assert _ff(torch, ff) == eff == (-1 if outcome == "ok" else W - 1)
    assert np.array_equal(got, exp)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["host", "device"])
@pytest.mark.parametrize("name,delta,outcome", CASES)
def test_hip_recombine_object_ragged(gpu, mode, name, delta, outcome):
    torch, A, ctx, F = gpu
    W, n = 1031, 4
    shares = [o[3] for o in _ragged(F, W, n, delta, seed=23)]
    args = shares if mode == "host" else [torch.from_numpy(s).cuda() for s in shares]
    if outcome == "range":
        with pytest.raises(A.AmphoraNativeError) as e:
            ctx.recombine_object(args)
        assert e.value.status == A._lib.AMPH_E_RANGE
        return
    got = ctx.recombine_object(args)
    got = got if mode == "host" else got.cpu().numpy()
    assert np.array_equal(got, F.recombine_object(shares))


@pytest.mark.gpu
def test_hip_ragged_device_accumulates(gpu):
    """AMPH_F_ACCUMULATE over a ragged call: an earlier (smaller) failing
    index already in first_fail stays; a fresh sentinel takes W-1."""
    torch, A, ctx, F = gpu
    import ctypes as C
    W, n = 4099, 2
    odos = _on(torch, "device", _ragged(F, W, n, -8, seed=31))
    arr, _ = ctx._odo_structs(odos)
    out = torch.empty((W, 16), dtype=torch.uint8, device="cuda")
    for start, want in ((NO_FAIL, W - 1), (17, 17)):
        ff = torch.full((1,), start, dtype=torch.int64, device="cuda")
        st = A._lib.lib.amph_recombine_verify(
            ctx._h, arr, n, out.data_ptr(), C.cast(C.c_void_p(ff.data_ptr()), C.POINTER(C.c_int64)),
            A._lib.AMPH_F_DEVICE | A._lib.AMPH_F_ACCUMULATE, C.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert st == 0
        torch.cuda.synchronize()
        assert int(ff.item()) == want


@pytest.mark.gpu
@pytest.mark.parametrize("name,delta,outcome", CASES)
def test_client_mirror_ragged_matches_the_reference(gpu, name, delta, outcome):
    """The Python client mirror (amphora_amd/client.py) hands each party's
    fields to the C ABI with their real byte lengths, so a ragged partner
    gives exactly the reference's outcome: the secrets, the
    IntegrityVerificationException whose message is built from the
    zero-padded word (copyOfRange), or the index exception -- compared with
    the oracle's verifyOutputDeliveryObjects / createSecret, message text
    included (the mirror used to cut the partial word and read
    past the short party's buffer when rendering the message)."""
    torch, A, ctx, F = gpu
    from amphora_amd import client as CL
    from amphora_amd.entities import IntegrityVerificationException, OutputDeliveryObject, Secret
    W, n = 37, 3
    odos = _ragged(F, W, n, delta, seed=41)
    util = O.ClientSecretShareUtil(P, R, RINV)
    pyodos = [O.OutputDeliveryObject(*[f.tobytes() for f in o]) for o in odos]
    codos = [OutputDeliveryObject(*[f.tobytes() for f in o]) for o in odos]
    cutil = CL.SecretShareUtil(ctx)
    secrets = [int.from_bytes(w.tobytes(), "little") for w in F.synth_words(seed=42, count=W - 2, mont=False)]
    for run_ref, run_mirror in (
            (lambda: O.verify_output_delivery_objects(util, pyodos),
             lambda: CL.verify_output_delivery_objects(cutil, codos)),
            (lambda: O.create_secret_masked_inputs(util, secrets, pyodos),
             lambda: CL.create_masked_input(cutil, Secret.of([], secrets), codos))):
        if outcome == "range":
            with pytest.raises(O.ArrayIndexOutOfBoundsException):
                run_ref()
            with pytest.raises(IndexError):
                run_mirror()
            continue
        if outcome == "pad":
            with pytest.raises(O.IntegrityVerificationException) as ref:
                run_ref()
            with pytest.raises(IntegrityVerificationException) as got:
                run_mirror()
            assert str(got.value) == str(ref.value)
            continue
        ref = run_ref()
        got = run_mirror()
        if isinstance(got, list):  # canonical secrets
            assert got == ref
        else:  # MaskedInput: its words equal the oracle's maskInput bytes
            assert [bytes(w) for w in got.data.words] == [bytes(x) for x in ref]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["host", "device"])
@pytest.mark.parametrize("name,delta,outcome", CASES)
def test_hip_mask_input_ragged_more_secrets_than_masks(gpu, mode, name, delta, outcome):
    """Ragged parties AND more secret words than masks: the outcome the
    reference reaches first -- copyOfRange's exception, then the MAC check
    over the zero-padded word, and only then the index error (createSecret,
    DefaultAmphoraClient.java:153-160) -- as AMPH_E_RANGE / AMPH_E_VERIFY
    (first_fail W-1) / AMPH_E_LEN, against the oracle."""
    torch, A, ctx, F = gpu
    W, n = 37, 3
    odos = _ragged(F, W, n, delta, seed=43)
    secrets = F.synth_words(seed=44, count=W + 5, mont=False)
    util = O.ClientSecretShareUtil(P, R, RINV)
    pyodos = [O.OutputDeliveryObject(*[f.tobytes() for f in o]) for o in odos]
    vals = [int.from_bytes(w.tobytes(), "little") for w in secrets]
    try:
        O.create_secret_masked_inputs(util, vals, pyodos)
        want = "none"
    except O.ArrayIndexOutOfBoundsException:
        want = "range"
    except O.IntegrityVerificationException:
        want = "verify"
    except IndexError:
        want = "len"
    assert want == {"range": "range", "pad": "verify", "ok": "len"}[outcome]
    args = _on(torch, mode, odos)
    sec = secrets if mode == "host" else torch.from_numpy(secrets).cuda()
    if want == "verify":
        _, ff = ctx.mask_input(args, sec)
        assert _ff(torch, ff) == W - 1
    else:
        with pytest.raises(A.AmphoraNativeError) as e:
            ctx.mask_input(args, sec)
        assert e.value.status == (A._lib.AMPH_E_RANGE if want == "range" else A._lib.AMPH_E_LEN)
