"""AMPH_F_HOST_IO through the plain C ABI (include/amphora.h): word arrays
passed as amph_host_array descriptors whose read / write callbacks the
library's staging threads call per batch -- what the JNI layer does with
Get/SetByteArrayRegion, here with ctypes callbacks over numpy arrays.

* amph_convert_share: the arrays are descriptors, the MAC key stays raw
  16 bytes (the header's list of raw arguments);
* amph_recombine_verify / amph_mask_input / amph_recombine_object with a
  ragged partner (recombineObject's copyOfRange semantics): the last word's
  partial bytes are read through the callback, never past the array's end.
Every result is compared with the C oracle.
"""
import ctypes as C

import numpy as np
import pytest

from oracle import amphora_oracle as O
from oracle import coracle

pytestmark = pytest.mark.gpu

P, R, RINV = O.TEST_PRIME, O.TEST_R, O.TEST_RINV
AMPH_F_HOST_IO = 0x4

RW = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p)


class _Desc(C.Structure):
    _fields_ = [("read", RW), ("write", RW), ("user", C.c_void_p)]


class HostArray:
    """One amph_host_array over a numpy uint8 buffer; callbacks bounds-check
    every request (a read past the end fails the call, as a JNI region copy
    would throw)."""

    def __init__(self, arr):
        self.arr = np.ascontiguousarray(arr, dtype=np.uint8).reshape(-1)
        self.reads = self.writes = 0
        self.out_of_range = 0

        def rd(_a, off, n, dst):
            if off + n > self.arr.size:
                self.out_of_range += 1
                return -1
            C.memmove(dst, self.arr.ctypes.data + off, n)
            self.reads += 1
            return 0

        def wr(_a, off, n, src):
            if off + n > self.arr.size:
                self.out_of_range += 1
                return -1
            C.memmove(self.arr.ctypes.data + off, src, n)
            self.writes += 1
            return 0

        self._rd, self._wr = RW(rd), RW(wr)
        self.desc = _Desc(self._rd, self._wr, None)

    @property
    def ptr(self):
        return C.addressof(self.desc)


@pytest.fixture(scope="module")
def env():
    import torch
    import amphora_amd as A
    assert torch.cuda.is_available()
    ctx = A.Context(P, R, RINV, device=0)
    ctx.set_batch_words(1 << 16)  # several batches per call: the staging threads run the callbacks
    return A, ctx, coracle.test_field(threads=16)


def test_convert_share_host_io_key_stays_raw(env):
    A, ctx, F = env
    W = 200_003
    masked = F.synth_words(seed=4, count=W)
    tuples = F.synth_words(seed=5, count=2 * W).reshape(W, 32)
    key = 0x1234_5678_9ABC_DEF0_0FED_CBA9_8765_4321 % P
    exp = F.convert_share(masked, tuples, key, False)
    hm, ht, ho = HostArray(masked), HostArray(tuples), HostArray(np.zeros((W, 32), np.uint8))
    st = A._lib.lib.amph_convert_share(ctx._h, hm.ptr, ht.ptr, W, key.to_bytes(16, "little"), 0, ho.ptr,
                                       AMPH_F_HOST_IO, None)
    assert st == 0, A._lib.lib.amph_last_error()
    assert np.array_equal(ho.arr.reshape(W, 32), exp)
    assert hm.reads > 1 and ho.writes > 1 and hm.out_of_range == ho.out_of_range == 0


def _odo_array(A, descs, lens, n):
    arr = (A._lib._AmphOdo * n)()
    for j in range(n):
        arr[j] = A._lib._AmphOdo(*[descs[j][k].ptr for k in range(5)], lens[j])
    return arr


@pytest.mark.parametrize("delta,outcome", [(37, "ok"), (-8, "pad"), (-16, "pad"), (-32, "range")])
def test_ragged_parties_host_io(env, delta, outcome):
    from tests.test_ragged_parties import _ragged
    A, ctx, F = env
    W, n = 150_001, 3
    odos = _ragged(F, W, n, delta, seed=5)
    descs = [[HostArray(f) for f in o] for o in odos]
    lens = [o[0].size for o in odos]
    arr = _odo_array(A, descs, lens, n)
    out = HostArray(np.zeros((W, 16), np.uint8))
    ff = C.c_int64(-1)
    st = A._lib.lib.amph_recombine_verify(ctx._h, arr, n, out.ptr, C.byref(ff), AMPH_F_HOST_IO, None)
    if outcome == "range":
        assert st == A._lib.AMPH_E_RANGE
        assert out.writes == 0
        return
    ey, eff = F.recombine_verify_object(odos)
    assert st == (0 if eff < 0 else A._lib.AMPH_E_VERIFY) and ff.value == eff
    assert np.array_equal(out.arr.reshape(W, 16), ey)
    secrets = F.synth_words(seed=6, count=W, mont=False)
    hs, hm = HostArray(secrets), HostArray(np.zeros((W, 16), np.uint8))
    ff = C.c_int64(-1)
    st = A._lib.lib.amph_mask_input(ctx._h, arr, n, hs.ptr, W, hm.ptr, C.byref(ff), AMPH_F_HOST_IO, None)
    em, mff = F.mask_input_object(secrets, odos)
    assert ff.value == mff and np.array_equal(hm.arr.reshape(W, 16), em)
    sh = (C.c_void_p * n)(*[descs[j][2].ptr for j in range(n)])
    nb = (C.c_size_t * n)(*lens)
    ho = HostArray(np.zeros((W, 16), np.uint8))
    assert A._lib.lib.amph_recombine_object(ctx._h, sh, n, nb, ho.ptr, AMPH_F_HOST_IO, None) == 0
    assert np.array_equal(ho.arr.reshape(W, 16), F.recombine_object([o[2] for o in odos]))
    for d in [x for ds in descs for x in ds] + [out, hs, hm, ho]:
        assert d.out_of_range == 0, "a callback was asked for bytes past its array's end"


def test_failed_callback_leaves_nothing_in_flight(env):
    """a read callback that fails part-way through a batched call
    (batches before it already copied in, their kernels and copies out
    queued) makes the call return AMPH_E_PARAM only after the pipeline's
    streams have drained (run_batched synchronises them on every error), so
    the next call -- which reuses the same page-locked staging slots -- gets
    exact results."""
    A, ctx, F = env
    W, n = 1 << 20, 2
    odos, _ = F.synth_odos(seed=41, n=n, W=W)
    good = [[HostArray(f) for f in o] for o in odos]
    lens = [o[0].nbytes for o in odos]
    bad = [[HostArray(f) for f in o] for o in odos]
    calls = {"n": 0}
    orig = bad[1][3]._rd

    def flaky(a, off, nb, dst):  # party 1's w field: the 3rd read fails
        calls["n"] += 1
        return -1 if calls["n"] == 3 else orig(a, off, nb, dst)
    bad[1][3]._rd2 = RW(flaky)
    bad[1][3].desc = _Desc(bad[1][3]._rd2, bad[1][3]._wr, None)
    out = HostArray(np.zeros((W, 16), np.uint8))
    ff = C.c_int64(-1)
    st = A._lib.lib.amph_recombine_verify(ctx._h, _odo_array(A, bad, lens, n), n, out.ptr, C.byref(ff),
                                          AMPH_F_HOST_IO, None)
    assert st == A._lib.AMPH_E_PARAM and calls["n"] >= 3
    out2 = HostArray(np.zeros((W, 16), np.uint8))
    ff = C.c_int64(-1)
    st = A._lib.lib.amph_recombine_verify(ctx._h, _odo_array(A, good, lens, n), n, out2.ptr, C.byref(ff),
                                          AMPH_F_HOST_IO, None)
    ey, eff = F.recombine_verify(odos)
    assert st == 0 and ff.value == eff == -1
    assert np.array_equal(out2.arr.reshape(W, 16), ey)
