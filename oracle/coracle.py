"""ctypes wrapper of the C oracle (oracle/amphora_oracle.c).

TEST INFRASTRUCTURE ONLY -- see the header of amphora_oracle.c.  Arrays are
numpy uint8 buffers; a "word array" is shape (W, 16).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_build", "libamphora_oracle.so")


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        vp, sz, i32, i64, u64 = C.c_void_p, C.c_size_t, C.c_int, C.c_int64, C.c_uint64
        pp = C.POINTER(C.c_void_p)
        L.orc_field_new.restype = vp
        L.orc_field_new.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.POINTER(C.c_int)]
        L.orc_field_free.argtypes = [vp]
        L.orc_recombine.argtypes = [vp, i32, pp, sz, vp, i32]
        L.orc_recombine_verify.restype = i64
        L.orc_recombine_verify.argtypes = [vp, i32, pp, pp, pp, pp, pp, sz, vp, i32]
        L.orc_mask_input.restype = i64
        L.orc_mask_input.argtypes = [vp, i32, pp, pp, pp, pp, pp, vp, sz, vp, i32]
        L.orc_convert_share.argtypes = [vp, vp, vp, C.c_char_p, i32, sz, vp, i32]
        L.orc_odo_pre.argtypes = [vp, vp, i32, vp, vp, sz, vp, vp, vp, vp, vp, i32]
        L.orc_recombine_diffs.argtypes = [vp, i32, pp, pp, sz, vp, i32]
        L.orc_odo_post.argtypes = [vp, vp, vp, i32, sz, vp, vp, i32]
        L.orc_synth_odos.argtypes = [vp, u64, i32, sz, pp, vp, i64, i32, i32]
        L.orc_synth_words.argtypes = [vp, u64, sz, vp, i32, i32]
        L.orc_max_threads.restype = i32
        _lib = L
    return _lib


def _ptrs(arrays):
    arr = (C.c_void_p * len(arrays))(*[a.ctypes.data for a in arrays])
    return C.cast(arr, C.POINTER(C.c_void_p)), arr


def _le16(x: int) -> bytes:
    return int(x).to_bytes(16, "little")


def default_threads() -> int:
    return int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))


def java_words(buf, W: int):
    """A party's byte[] as the W words recombineObject reads from it (client
    SecretShareUtil.java:87-88): word i = Arrays.copyOfRange(buf, 16 i,
    16 i + 16) -- amphora_oracle.copy_of_range, vectorised: cut past 16 W,
    zero-padded past the end, ArrayIndexOutOfBoundsException when some word
    i < W starts past the end (16 i > len).  Returns a (W, 16) uint8 array."""
    from oracle.amphora_oracle import ArrayIndexOutOfBoundsException
    a = np.frombuffer(bytes(buf), np.uint8) if isinstance(buf, (bytes, bytearray)) else \
        np.ascontiguousarray(buf, dtype=np.uint8).reshape(-1)
    if W and 16 * (W - 1) > a.size:
        raise ArrayIndexOutOfBoundsException(
            "arraycopy: word %d starts past the end of byte[%d]" % (a.size // 16 + 1, a.size))
    out = np.zeros((W, 16), np.uint8)
    k = min(a.size, 16 * W)
    out.reshape(-1)[:k] = a[:k]
    return out


class Field:
    """One prime field; mirrors MpSpdzIntegrationUtils.of(prime, r, rInv)."""

    def __init__(self, prime: int, r: int, r_inv: int, threads: int | None = None):
        self.prime, self.r, self.r_inv = prime, r, r_inv
        st = C.c_int(0)
        self._f = lib().orc_field_new(_le16(prime), _le16(r), _le16(r_inv), C.byref(st))
        if st.value != 0:
            raise ValueError("invalid field parameters (status %d)" % st.value)
        self.threads = threads or default_threads()

    def __del__(self):
        if getattr(self, "_f", None) and _lib is not None:
            _lib.orc_field_free(self._f)
            self._f = None

    # -- client ------------------------------------------------------------
    def recombine(self, shares):
        W = shares[0].shape[0]
        out = np.empty((W, 16), np.uint8)
        p, keep = _ptrs(shares)
        lib().orc_recombine(self._f, len(shares), p, W, out.ctypes.data, self.threads)
        return out

    def recombine_verify(self, odos):
        """odos: list over parties of 5-tuples (y, r, v, w, u) of (W,16) arrays.
        Returns (canonical secrets (W,16) LE, first_fail or -1)."""
        n = len(odos)
        W = odos[0][0].shape[0]
        fl = [_ptrs([odos[j][k] for j in range(n)]) for k in range(5)]
        out = np.empty((W, 16), np.uint8)
        ff = lib().orc_recombine_verify(self._f, n, *[x[0] for x in fl], W, out.ctypes.data,
                                        self.threads)
        return out, ff

    def mask_input(self, secrets16, mask_odos):
        n = len(mask_odos)
        W = secrets16.shape[0]
        fl = [_ptrs([mask_odos[j][k] for j in range(n)]) for k in range(5)]
        out = np.empty((W, 16), np.uint8)
        ff = lib().orc_mask_input(self._f, n, *[x[0] for x in fl],
                                  np.ascontiguousarray(secrets16).ctypes.data, W,
                                  out.ctypes.data, self.threads)
        return out, ff

    # -- recombineObject over parties of their own lengths ---------------------
    def recombine_object(self, shares):
        """recombineObject (SecretShareUtil.java:70-90): W = party 0's length
        // 16, every party's words read as java_words does."""
        if len(shares) == 0:
            return np.empty((0, 16), np.uint8)
        W = len(bytes(shares[0])) // 16 if isinstance(shares[0], (bytes, bytearray)) else \
            np.asarray(shares[0]).nbytes // 16
        return self.recombine([java_words(s, W) for s in shares])

    def _java_odos(self, odos):
        W = np.asarray(odos[0][0]).nbytes // 16
        return [tuple(java_words(f, W) for f in o) for o in odos], W

    def recombine_verify_object(self, odos):
        """verifyOutputDeliveryObjects (DefaultAmphoraClient.java:476-505) over
        byte[] fields of any length: the five recombineObject calls take
        party 0's word count and copyOfRange semantics."""
        jo, _ = self._java_odos(odos)
        return self.recombine_verify(jo)

    def mask_input_object(self, secrets16, mask_odos):
        """createSecret (:150-160) over byte[] mask fields of any length:
        verify every mask word, mask the len(secrets16) <= W first ones.
        Returns (masked, first failing mask index or -1)."""
        jo, W = self._java_odos(mask_odos)
        _, ff = self.recombine_verify(jo)
        S = secrets16.shape[0]
        m, _ = self.mask_input(secrets16, [tuple(f[:S] for f in o) for o in jo])
        return m, ff

    # -- service -----------------------------------------------------------
    def convert_share(self, masked16, tuples32, mac_key: int, use_zero_input: bool):
        W = masked16.shape[0]
        out = np.empty((W, 32), np.uint8)
        lib().orc_convert_share(self._f, masked16.ctypes.data, tuples32.ctypes.data,
                                _le16(mac_key % self.prime), int(use_zero_input), W,
                                out.ctypes.data, self.threads)
        return out

    def odo_pre(self, share_data, share_stride, masks32, triples96):
        W = share_data.shape[0]
        y, r, v = (np.empty((W, 16), np.uint8) for _ in range(3))
        mag = np.empty((2 * W, 2, 16), np.uint8)
        neg = np.empty((2 * W, 2), np.uint8)
        lib().orc_odo_pre(self._f, share_data.ctypes.data, share_stride, masks32.ctypes.data,
                          triples96.ctypes.data, W, y.ctypes.data, r.ctypes.data,
                          v.ctypes.data, mag.ctypes.data, neg.ctypes.data, self.threads)
        return y, r, v, mag, neg

    def recombine_diffs(self, mags, negs):
        nvals = mags[0].shape[0] * 2
        out = np.empty((nvals // 2, 2, 16), np.uint8)
        pm, k1 = _ptrs(mags)
        pn, k2 = _ptrs(negs)
        lib().orc_recombine_diffs(self._f, len(mags), pm, pn, nvals, out.ctypes.data,
                                  self.threads)
        return out

    def odo_post(self, opened, triples96, is_player0: bool):
        W = opened.shape[0] // 2
        w, u = np.empty((W, 16), np.uint8), np.empty((W, 16), np.uint8)
        lib().orc_odo_post(self._f, opened.ctypes.data, triples96.ctypes.data, int(is_player0),
                           W, w.ctypes.data, u.ctypes.data, self.threads)
        return w, u

    # -- synthetic inputs ----------------------------------------------------
    def synth_odos(self, seed: int, n: int, W: int, y_plain=None, fault_index: int = -1,
                   noncanon_permille: int = 0):
        """Honest N-party ODOs; returns list over parties of (y, r, v, w, u)."""
        bufs = np.empty((5, n, W, 16), np.uint8)
        arrs = [bufs[k, j] for k in range(5) for j in range(n)]
        p, keep = _ptrs(arrs)
        lib().orc_synth_odos(self._f, seed, n, W, p,
                             None if y_plain is None else np.ascontiguousarray(y_plain).ctypes.data,
                             fault_index, noncanon_permille, self.threads)
        return [tuple(bufs[k, j] for k in range(5)) for j in range(n)], bufs

    def synth_words(self, seed: int, count: int, mont: bool = True):
        out = np.empty((count, 16), np.uint8)
        lib().orc_synth_words(self._f, seed, count, out.ctypes.data, int(mont), self.threads)
        return out


def test_field(threads=None) -> Field:
    from .amphora_oracle import TEST_PRIME, TEST_R, TEST_RINV
    return Field(TEST_PRIME, TEST_R, TEST_RINV, threads)
