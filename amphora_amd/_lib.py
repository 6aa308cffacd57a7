"""ctypes binding of libamphora_hip.so (the C ABI in include/amphora.h).

This is the product path: every arithmetic call goes to the HIP kernels.
There is no CPU fallback -- if the shared library is missing or cannot be
loaded, importing this module raises.

Buffers: host calls take C-contiguous numpy uint8 arrays (or bytes); device
calls take torch uint8 tensors on the context's GPU and run asynchronously on
torch's current stream (so torch.cuda.Event timing sees them).
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libamphora_hip.so")

AMPH_OK, AMPH_E_VERIFY, AMPH_E_LEN, AMPH_E_PARAM, AMPH_E_HIP, AMPH_E_NOMEM, AMPH_E_RANGE = 0, 1, 2, 3, 4, 5, 6
AMPH_F_DEVICE = 1
AMPH_F_ACCUMULATE = 2
AMPH_NO_FAILURE = 0x7F7F7F7F7F7F7F7F
MAX_PARTIES = 16


class AmphoraNativeError(RuntimeError):
    def __init__(self, status: int, detail: str):
        super().__init__("%s (status %d): %s" % (_STATUS.get(status, "error"), status, detail))
        self.status = status


def _need(cond: bool, detail: str):
    """Host-side length check of a call whose C entry point takes raw pointers
    and one word count (it cannot see the buffers' sizes)."""
    if not cond:
        raise AmphoraNativeError(AMPH_E_LEN, detail)


_STATUS = {AMPH_E_VERIFY: "verification failed", AMPH_E_LEN: "length invariant",
           AMPH_E_PARAM: "invalid argument", AMPH_E_HIP: "HIP error", AMPH_E_NOMEM: "out of memory",
           AMPH_E_RANGE: "array index out of range"}


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError("libamphora_hip.so not built (%s): run `python tools/build_native.py` "
                          "or __graft_entry__.build(); there is no CPU fallback" % LIB_PATH)
    # torch (if present) ships its own libamdhip64.so.7; loading it first makes
    # this library bind to the same HIP runtime instance (same SONAME), so
    # device pointers and streams from torch are valid here.
    if "torch" not in sys.modules:
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    L = C.CDLL(LIB_PATH)
    vp, sz, i32, u32, u64, i64p = C.c_void_p, C.c_size_t, C.c_int, C.c_uint32, C.c_uint64, C.POINTER(C.c_int64)
    L.amph_ctx_create.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, i32, C.POINTER(vp)]
    L.amph_ctx_create_multi.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.POINTER(i32), i32,
                                        C.POINTER(vp)]
    L.amph_ctx_device_count.argtypes = [vp]
    L.amph_ctx_destroy.argtypes = [vp]
    L.amph_ctx_device.argtypes = [vp]
    L.amph_ctx_set_batch_words.argtypes = [vp, sz]
    L.amph_ctx_stats.argtypes = [vp, vp]
    L.amph_strerror.restype = C.c_char_p
    L.amph_strerror.argtypes = [i32]
    L.amph_last_error.restype = C.c_char_p
    L.amph_version.restype = C.c_char_p
    L.amph_build_id.restype = C.c_char_p
    L.amph_recombine_verify.argtypes = [vp, vp, i32, vp, i64p, u32, vp]
    L.amph_mask_input.argtypes = [vp, vp, i32, vp, sz, vp, i64p, u32, vp]
    L.amph_recombine.argtypes = [vp, C.POINTER(vp), i32, sz, vp, u32, vp]
    L.amph_recombine_object.argtypes = [vp, C.POINTER(vp), i32, C.POINTER(sz), vp, u32, vp]
    L.amph_verify.argtypes = [vp, vp, vp, vp, vp, vp, sz, i64p, u32, vp]
    L.amph_verify_message.argtypes = [vp, vp, vp, vp, vp, vp, C.c_char_p, sz]
    L.amph_mask_words.argtypes = [vp, vp, vp, sz, vp, u32, vp]
    L.amph_mask_word_host.argtypes = [vp, C.c_char_p, C.c_char_p, vp]
    L.amph_to_gfp.argtypes = [vp, vp, sz, vp, u32, vp]
    L.amph_from_gfp.argtypes = [vp, vp, sz, vp, u32, vp]
    L.amph_convert_share.argtypes = [vp, vp, vp, sz, C.c_char_p, i32, vp, u32, vp]
    L.amph_odo_pre.argtypes = [vp, vp, sz, vp, vp, sz, vp, vp, vp, vp, vp, u32, vp]
    L.amph_open_diffs.argtypes = [vp, C.POINTER(vp), C.POINTER(vp), i32, sz, vp, u32, vp]
    L.amph_odo_post.argtypes = [vp, vp, vp, sz, i32, vp, vp, u32, vp]
    L.amph_open_post.argtypes = [vp, C.POINTER(vp), C.POINTER(vp), i32, vp, sz, i32, vp, vp, u32, vp]
    L.amph_host_register.argtypes = [vp, vp, sz]
    L.amph_host_unregister.argtypes = [vp, vp]
    L.amph_time_next_launch.argtypes = [vp, vp]
    L.amph_timing_event_create.argtypes = [C.POINTER(vp)]
    L.amph_timing_event_destroy.argtypes = [vp]
    L.amph_timing_event_record.argtypes = [vp, vp]
    L.amph_timing_event_elapsed_ms.argtypes = [vp, vp, C.POINTER(C.c_float)]
    L.amph_base64_encode.argtypes = [vp, vp, sz, vp, u32, vp]
    L.amph_base64_decode.argtypes = [vp, vp, sz, vp, C.POINTER(C.c_size_t), i64p, u32, vp]
    L.amph_base64_encode_words.argtypes = [vp, vp, sz, vp, u32, vp]
    L.amph_base64_decode_words.argtypes = [vp, vp, sz, vp, i64p, u32, vp]
    L.amph_exchange_max_chars.restype = sz
    L.amph_exchange_max_chars.argtypes = [sz]
    L.amph_exchange_encode.argtypes = [vp, vp, vp, sz, vp, sz, vp, u32, vp]
    L.amph_exchange_decode.argtypes = [vp, vp, sz, sz, vp, vp, i64p, u32, vp]
    L.amph_synth_odos.argtypes = [vp, u64, i32, sz, C.POINTER(vp), vp, C.c_int64, i32, vp]
    L.amph_synth_words.argtypes = [vp, u64, sz, vp, vp]
    L.amph_stream_probe.argtypes = [vp, vp, i32, vp, sz, vp, vp]
    L.amph_recombine_verify_b64.argtypes = [vp, vp, i32, sz, vp, i64p, i64p, u32, vp]
    L.amph_mask_input_b64.argtypes = [vp, vp, i32, sz, vp, sz, vp, vp, i64p, i64p, u32, vp]
    L.amph_party_begin.argtypes = [vp, vp, sz, vp, vp, sz, i32, vp, vp, vp, C.POINTER(vp)]
    L.amph_party_words.restype = sz
    L.amph_party_words.argtypes = [vp]
    L.amph_party_text_len.restype = u64
    L.amph_party_text_len.argtypes = [vp]
    L.amph_party_text.argtypes = [vp, vp, sz]
    L.amph_party_partner.argtypes = [vp, i32, vp, sz, i64p]
    L.amph_party_finish.argtypes = [vp, i32, vp, vp]
    L.amph_party_finish_b64.argtypes = [vp, i32, C.POINTER(vp)]
    L.amph_party_free.restype = None
    L.amph_party_free.argtypes = [vp]
    L.amph_party_begin_dev.argtypes = [vp, vp, sz, vp, vp, sz, i32, vp, vp, vp, vp, C.POINTER(vp)]
    L.amph_party_text_dev.argtypes = [vp, C.POINTER(vp), C.POINTER(vp)]
    L.amph_party_partner_dev.argtypes = [vp, i32, vp, sz, vp, vp]
    L.amph_party_finish_b64_dev.argtypes = [vp, i32, C.POINTER(vp), vp]
    L.amph_party_reset_partner.argtypes = [vp, i32]
    return L


lib = _load()


def build_id() -> str:
    """The id compiled into the loaded library (amph_build_id)."""
    return lib.amph_build_id().decode()


def tree_build_id() -> str:
    """The id of the source tree beside the library (tools/build_native.py
    tree_digest over the same sources, headers, flags and arch)."""
    root = os.path.dirname(HERE)
    sys.path.insert(0, os.path.join(root, "tools"))
    try:
        import build_native
    finally:
        sys.path.pop(0)
    return build_native.tree_digest()


def check_build_id() -> str:
    """Raise unless the loaded library was built from this tree; returns the id."""
    got, want = build_id(), tree_build_id()
    if got != want:
        raise RuntimeError("libamphora_hip.so carries build id %s but the sources beside it hash to %s: "
                           "rebuild (__graft_entry__.build())" % (got, want))
    return got

EXPORTED = ["amph_ctx_create", "amph_ctx_create_multi", "amph_ctx_device_count",
            "amph_ctx_destroy", "amph_ctx_device", "amph_ctx_set_batch_words", "amph_ctx_stats", "amph_strerror",
            "amph_last_error", "amph_version", "amph_build_id", "amph_recombine_verify", "amph_mask_input",
            "amph_recombine", "amph_recombine_object", "amph_verify", "amph_verify_message", "amph_mask_words", "amph_mask_word_host",
            "amph_to_gfp", "amph_from_gfp", "amph_convert_share", "amph_odo_pre",
            "amph_open_diffs", "amph_odo_post", "amph_open_post", "amph_synth_odos", "amph_synth_words",
            "amph_host_register", "amph_host_unregister", "amph_time_next_launch",
            "amph_timing_event_create", "amph_timing_event_destroy", "amph_timing_event_record",
            "amph_timing_event_elapsed_ms", "amph_base64_encode", "amph_base64_decode",
            "amph_base64_encode_words", "amph_base64_decode_words", "amph_exchange_max_chars",
            "amph_exchange_encode", "amph_exchange_decode", "amph_stream_probe",
            "amph_recombine_verify_b64", "amph_mask_input_b64", "amph_party_begin", "amph_party_words", "amph_party_text_len",
            "amph_party_text", "amph_party_partner", "amph_party_finish", "amph_party_finish_b64",
            "amph_party_free", "amph_party_begin_dev", "amph_party_text_dev", "amph_party_partner_dev",
            "amph_party_finish_b64_dev", "amph_party_reset_partner"]


class TimingEvent:
    """A timing-only hipEvent_t (amph_timing_event_create: no system-scope
    fence on record) for amph_time_next_launch."""

    def __init__(self):
        h = C.c_void_p()
        Context._check(lib.amph_timing_event_create(C.byref(h)))
        self.handle = h

    def elapsed_ms(self, stop: "TimingEvent") -> float:
        ms = C.c_float()
        Context._check(lib.amph_timing_event_elapsed_ms(self.handle, stop.handle, C.byref(ms)))
        return ms.value

    def __del__(self):
        if getattr(self, "handle", None) is not None and lib is not None:
            lib.amph_timing_event_destroy(self.handle)
            self.handle = None


class _AmphOdo(C.Structure):
    _fields_ = [("secret_shares", C.c_void_p), ("r_shares", C.c_void_p), ("v_shares", C.c_void_p),
                ("w_shares", C.c_void_p), ("u_shares", C.c_void_p), ("nbytes", C.c_size_t)]


class _AmphStats(C.Structure):  # amph_stats
    _fields_ = [(k, C.c_uint64) for k in ("kernel_launches", "pool_buffers", "pool_bytes",
                                           "device_workers", "worker_tasks")]


class _AmphOdoB64(C.Structure):  # amph_odo_b64: one party's five base64 field texts
    _fields_ = [("secret_shares", C.c_void_p), ("r_shares", C.c_void_p), ("v_shares", C.c_void_p),
                ("w_shares", C.c_void_p), ("u_shares", C.c_void_p), ("nchars", C.c_size_t)]


def le16(x: int) -> bytes:
    return int(x).to_bytes(16, "little")


def _is_dev(x) -> bool:
    return hasattr(x, "is_cuda") and x.is_cuda


def words_view(x, width: int = 16):
    """bytes / bytearray / numpy -> C-contiguous uint8 numpy array (n, width)."""
    if _is_dev(x):
        return x
    if isinstance(x, (bytes, bytearray, memoryview)):
        a = np.frombuffer(bytes(x), np.uint8)
    else:
        a = np.ascontiguousarray(x, dtype=np.uint8)
    n = a.size // width
    return a.reshape(-1)[: n * width].reshape(n, width)


def byte_len(x) -> int:
    """Length in bytes of a word buffer as the caller passed it (a ragged
    party's array need not hold whole words)."""
    if _is_dev(x):
        return x.numel() * x.element_size()
    if isinstance(x, (bytes, bytearray, memoryview)):
        return memoryview(x).nbytes
    # the same conversion words_view makes: the length of the uint8 buffer whose
    # pointer goes to C (an int64 array is 8x its converted size in nbytes)
    return int(np.ascontiguousarray(x, dtype=np.uint8).size)


def _ptr(x):
    if x is None:
        return None
    if _is_dev(x):
        return x.data_ptr()
    return x.ctypes.data


class Context:
    """One amph_ctx: field parameters (prime, r, rInv) bound to one GPU."""

    def __init__(self, prime: int, r: int, r_inv: int, device: int = 0, devices=None):
        """devices: several GPU ordinals -> amph_ctx_create_multi (host-pointer
        calls are sharded over them); device-pointer calls use devices[0]."""
        if devices is not None and len(devices) > 0:
            device = int(devices[0])
        self.prime, self.r, self.r_inv, self.device = prime, r, r_inv, device
        h = C.c_void_p()
        keys = (le16(prime % (1 << 128)), le16(r % (1 << 128)), le16(r_inv % (1 << 128)))
        if devices is not None and len(devices) > 1:
            arr = (C.c_int * len(devices))(*[int(d) for d in devices])
            self._check(lib.amph_ctx_create_multi(*keys, arr, len(devices), C.byref(h)))
        else:
            self._check(lib.amph_ctx_create(*keys, device, C.byref(h)))
        self._h = h

    @property
    def device_count(self) -> int:
        return lib.amph_ctx_device_count(self._h)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib.amph_ctx_destroy(h)
            self._h = None

    @staticmethod
    def _check(st: int, allow_verify: bool = False):
        if st == AMPH_OK or (allow_verify and st == AMPH_E_VERIFY):
            return st
        raise AmphoraNativeError(st, lib.amph_last_error().decode())

    def stats(self) -> dict:
        """amph_ctx_stats: kernel launches, pooled party buffers, device workers."""
        st = _AmphStats()
        self._check(lib.amph_ctx_stats(self._h, C.byref(st)))
        return {k: int(getattr(st, k)) for k, _ in _AmphStats._fields_}

    def set_batch_words(self, words: int):
        self._check(lib.amph_ctx_set_batch_words(self._h, words))

    def host_register(self, array: np.ndarray):
        """Page-lock a numpy buffer so host-pointer calls DMA it directly."""
        self._check(lib.amph_host_register(self._h, array.ctypes.data, array.nbytes))

    def host_unregister(self, array: np.ndarray):
        self._check(lib.amph_host_unregister(self._h, array.ctypes.data))

    # -- mode plumbing ----------------------------------------------------------
    def _mode(self, *arrays):
        dev = [_is_dev(a) for a in arrays if a is not None]
        if any(dev) and not all(dev):
            raise ValueError("mix of host and device buffers")
        if dev and dev[0]:
            import torch
            return AMPH_F_DEVICE, C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        return 0, None

    def _empty(self, like, shape, dtype="uint8"):
        if _is_dev(like):
            import torch
            return torch.empty(shape, dtype=getattr(torch, dtype), device=like.device)
        return np.empty(shape, dtype=dtype)

    def _ff(self, like):
        if _is_dev(like):
            import torch
            t = torch.empty(1, dtype=torch.int64, device=like.device)
            return t, C.cast(C.c_void_p(t.data_ptr()), C.POINTER(C.c_int64))
        v = C.c_int64(-1)
        return v, C.pointer(v)

    @staticmethod
    def _ff_value(ff):
        if isinstance(ff, C.c_int64):
            return ff.value
        return ff  # device tensor: AMPH_NO_FAILURE or index, read by the caller

    def _odo_structs(self, odos):
        n = len(odos)
        arr = (_AmphOdo * n)()
        views = []
        for j, o in enumerate(odos):
            lens = [byte_len(f) for f in o]
            if len(lens) != 5 or any(b != lens[0] for b in lens):
                # OutputDeliveryObject's constructor invariant (OutputDeliveryObject.java:90-96)
                raise AmphoraNativeError(AMPH_E_LEN, "The provided shares must be of the same length")
            fs = [words_view(f) for f in o]
            views.append(fs)
            # the party's own byte length: parties may differ (recombineObject's
            # ragged semantics, include/amphora.h amph_odo)
            arr[j] = _AmphOdo(*[_ptr(f) for f in fs], lens[0])
        return arr, views

    def _out(self, like, shape, out):
        """A fresh output buffer, or the caller's `out` (same memory kind,
        C-contiguous uint8 of exactly `shape`) so repeated calls reuse one
        (page-locked, if the caller registered it) buffer."""
        if out is None:
            return self._empty(like, shape)
        if _is_dev(out) != _is_dev(like):
            raise ValueError("out must live where the inputs live")
        ok = (tuple(out.shape) == tuple(shape) and str(out.dtype).endswith("uint8") and
              (out.is_contiguous() if _is_dev(out) else out.flags["C_CONTIGUOUS"]))
        if not ok:
            raise ValueError("out must be a C-contiguous uint8 array of shape %r" % (shape,))
        return out

    # -- client --------------------------------------------------------------
    def recombine_verify(self, odos, out=None):
        """odos: list over parties of (y, r, v, w, u) word arrays.
        Returns (canonical secrets (W,16), first_fail) -- first_fail is -1 /
        index on the host path, an int64[1] device tensor on the device path."""
        arr, views = self._odo_structs(odos)
        flags, stream = self._mode(*[f for v in views for f in v])
        W = arr[0].nbytes // 16  # party 0's word count (SecretShareUtil.java:75)
        out = self._out(views[0][0], (W, 16), out)
        ff, ffp = self._ff(views[0][0])
        self._check(lib.amph_recombine_verify(self._h, arr, len(odos), _ptr(out), ffp, flags,
                                              stream), allow_verify=True)
        return out, self._ff_value(ff)

    def mask_input(self, mask_odos, secrets16, out=None):
        arr, views = self._odo_structs(mask_odos)
        s = words_view(secrets16)
        flags, stream = self._mode(s, *[f for v in views for f in v])
        out = self._out(s, (s.shape[0], 16), out)
        ff, ffp = self._ff(s)
        self._check(lib.amph_mask_input(self._h, arr, len(mask_odos), _ptr(s), s.shape[0],
                                        _ptr(out), ffp, flags, stream), allow_verify=True)
        return out, self._ff_value(ff)

    def recombine(self, shares):
        vs = [words_view(s) for s in shares]
        flags, stream = self._mode(*vs)
        W = vs[0].shape[0]
        out = self._empty(vs[0], (W, 16))
        ptrs = (C.c_void_p * len(vs))(*[_ptr(v) for v in vs])
        self._check(lib.amph_recombine(self._h, ptrs, len(vs), W * 16, _ptr(out), flags, stream))
        return out

    def recombine_object(self, shares):
        """recombineObject exactly (client SecretShareUtil.java:70-90): each
        party's share array of its own byte length (amph_recombine_object)."""
        if len(shares) == 0:
            return np.empty((0, 16), np.uint8)
        lens = (C.c_size_t * len(shares))(*[byte_len(s) for s in shares])
        vs = [words_view(s) for s in shares]
        flags, stream = self._mode(*vs)
        W = lens[0] // 16
        out = self._empty(vs[0], (W, 16))
        ptrs = (C.c_void_p * len(vs))(*[_ptr(v) for v in vs])
        self._check(lib.amph_recombine_object(self._h, ptrs, len(vs), lens, _ptr(out), flags, stream))
        return out

    def verify(self, y, r, u, v, w):
        a = [words_view(x) for x in (y, r, u, v, w)]
        flags, stream = self._mode(*a)
        ff, ffp = self._ff(a[0])
        self._check(lib.amph_verify(self._h, *[_ptr(x) for x in a], a[0].shape[0], ffp, flags,
                                    stream), allow_verify=True)
        return self._ff_value(ff)

    def verify_message(self, y: int, r: int, u: int, v: int, w: int) -> str:
        buf = C.create_string_buffer(1024)
        n = lib.amph_verify_message(self._h, *[le16(x) for x in (y, r, u, v, w)], buf, 1024)
        if n < 0:
            raise AmphoraNativeError(-n, lib.amph_last_error().decode())
        return buf.value.decode()

    def mask_words(self, secrets16, masks16):
        s, m = words_view(secrets16), words_view(masks16)
        flags, stream = self._mode(s, m)
        out = self._empty(s, (s.shape[0], 16))
        self._check(lib.amph_mask_words(self._h, _ptr(s), _ptr(m), s.shape[0], _ptr(out), flags,
                                        stream))
        return out

    def to_gfp(self, words16):
        a = words_view(words16)
        flags, stream = self._mode(a)
        out = self._empty(a, (a.shape[0], 16))
        self._check(lib.amph_to_gfp(self._h, _ptr(a), a.shape[0], _ptr(out), flags, stream))
        return out

    def from_gfp(self, words16):
        a = words_view(words16)
        flags, stream = self._mode(a)
        out = self._empty(a, (a.shape[0], 16))
        self._check(lib.amph_from_gfp(self._h, _ptr(a), a.shape[0], _ptr(out), flags, stream))
        return out

    # -- service -------------------------------------------------------------
    def convert_share(self, masked16, tuples32, mac_key: int, use_zero_input_as_data: bool):
        m, t = words_view(masked16), words_view(tuples32, 32)
        _need(t.shape[0] >= m.shape[0], "Received more input data than available inputMasks.")
        flags, stream = self._mode(m, t)
        out = self._empty(m, (m.shape[0], 32))
        self._check(lib.amph_convert_share(self._h, _ptr(m), _ptr(t), m.shape[0],
                                           le16(mac_key % self.prime), int(use_zero_input_as_data),
                                           _ptr(out), flags, stream))
        return out

    def odo_pre(self, share_data, share_stride: int, masks32, triples96):
        sd = words_view(share_data, share_stride)
        mk, tr = words_view(masks32, 32), words_view(triples96, 96)
        W = sd.shape[0]
        # 2 input masks and 2 triples per word (OutputDeliveryService.java:102-107,177-185)
        _need(mk.shape[0] == 2 * W, "expected %d input-mask tuples, got %d" % (2 * W, mk.shape[0]))
        _need(tr.shape[0] == 2 * W, "expected %d multiplication triples, got %d" % (2 * W, tr.shape[0]))
        flags, stream = self._mode(sd, mk, tr)
        y, r, v = (self._empty(sd, (W, 16)) for _ in range(3))
        mag = self._empty(sd, (2 * W, 2, 16))
        neg = self._empty(sd, (2 * W, 2))
        self._check(lib.amph_odo_pre(self._h, _ptr(sd), share_stride, _ptr(mk), _ptr(tr), W,
                                     _ptr(y), _ptr(r), _ptr(v), _ptr(mag), _ptr(neg), flags,
                                     stream))
        return y, r, v, mag, neg

    def open_diffs(self, mags, negs):
        ms = [m if _is_dev(m) else np.ascontiguousarray(m, np.uint8) for m in mags]
        ns = [n if _is_dev(n) else np.ascontiguousarray(n, np.uint8) for n in negs]
        _need(len(ms) == len(ns) and len(ms) >= 1, "one (mag, neg) pair per party")
        n_pairs = ms[0].shape[0]
        for m, n in zip(ms, ns):  # every party opens the same 2W pairs (recombineDiffs :231-272)
            _need(tuple(m.shape) == (n_pairs, 2, 16) and tuple(n.shape) == (n_pairs, 2),
                  "party diff lists differ in length: %s / %s vs %d pairs"
                  % (tuple(m.shape), tuple(n.shape), n_pairs))
        flags, stream = self._mode(*ms, *ns)
        out = self._empty(ms[0], (n_pairs, 2, 16))
        pm = (C.c_void_p * len(ms))(*[_ptr(x) for x in ms])
        pn = (C.c_void_p * len(ns))(*[_ptr(x) for x in ns])
        self._check(lib.amph_open_diffs(self._h, pm, pn, len(ms), n_pairs, _ptr(out), flags, stream))
        return out

    def odo_post(self, opened, triples96, is_player0: bool):
        op = opened if _is_dev(opened) else np.ascontiguousarray(opened, np.uint8)
        tr = words_view(triples96, 96)
        _need(tr.shape[0] % 2 == 0 and tuple(op.shape) == (tr.shape[0], 2, 16),
              "opened values %s do not match %d triples" % (tuple(op.shape), tr.shape[0]))
        flags, stream = self._mode(op, tr)
        W = tr.shape[0] // 2
        w, u = self._empty(tr, (W, 16)), self._empty(tr, (W, 16))
        self._check(lib.amph_odo_post(self._h, _ptr(op), _ptr(tr), W, int(is_player0), _ptr(w),
                                      _ptr(u), flags, stream))
        return w, u

    def open_post(self, mags, negs, triples96, is_player0: bool):
        """open_diffs + odo_post in one launch (amph_open_post): every party's
        signed diffs + the triples -> (w, u); the opened values stay on chip."""
        ms = [m if _is_dev(m) else np.ascontiguousarray(m, np.uint8) for m in mags]
        ns = [n if _is_dev(n) else np.ascontiguousarray(n, np.uint8) for n in negs]
        tr = words_view(triples96, 96)
        _need(len(ms) == len(ns) and len(ms) >= 1, "one (mag, neg) pair per party")
        n_pairs = tr.shape[0]
        _need(n_pairs % 2 == 0, "triples must be 2 per word")
        for m, n in zip(ms, ns):
            _need(tuple(m.shape) == (n_pairs, 2, 16) and tuple(n.shape) == (n_pairs, 2),
                  "party diff lists %s / %s do not match %d triples"
                  % (tuple(m.shape), tuple(n.shape), n_pairs))
        flags, stream = self._mode(tr, *ms, *ns)
        W = n_pairs // 2
        w, u = self._empty(tr, (W, 16)), self._empty(tr, (W, 16))
        pm = (C.c_void_p * len(ms))(*[_ptr(x) for x in ms])
        pn = (C.c_void_p * len(ns))(*[_ptr(x) for x in ns])
        self._check(lib.amph_open_post(self._h, pm, pn, len(ms), _ptr(tr), W, int(is_player0), _ptr(w),
                                       _ptr(u), flags, stream))
        return w, u

    # -- K_RV / K_MASK straight from the base64 wire text ----------------------
    def _text_structs(self, texts):
        """texts: per party the five field strings (str / bytes / uint8 arrays,
        or 16-byte-aligned uint8 device tensors) in ODO order."""
        arr = (_AmphOdoB64 * len(texts))()
        keep = []
        for j, t in enumerate(texts):
            if len(t) != 5:
                raise ValueError("five base64 fields per party")
            fs = []
            for x in t:
                if isinstance(x, str):
                    x = x.encode("ascii", errors="replace")
                if isinstance(x, (bytes, bytearray, memoryview)):
                    x = np.frombuffer(bytes(x), np.uint8)
                elif not _is_dev(x):
                    x = np.ascontiguousarray(x, np.uint8).reshape(-1)
                fs.append(x)
            lens = {(f.numel() if _is_dev(f) else f.size) for f in fs}
            if len(lens) != 1:
                raise AmphoraNativeError(AMPH_E_LEN, "The provided shares must be of the same length")
            keep.extend(fs)
            arr[j] = _AmphOdoB64(*[_ptr(f) for f in fs], lens.pop())
        return arr, keep

    def recombine_verify_b64(self, texts, words: int):
        """amph_recombine_verify_b64: (canonical secrets (W, 16), first_fail,
        bad_char).  Host: first_fail / bad_char are -1 or indices (a bad
        character raises ValueError); device: int64[1] tensors."""
        arr, keep = self._text_structs(texts)
        flags, stream = self._mode(*keep)
        out = self._empty(keep[0], (words, 16))
        ff, ffp = self._ff(keep[0])
        bad, badp = self._ff(keep[0])
        st = lib.amph_recombine_verify_b64(self._h, arr, len(texts), words, _ptr(out), ffp, badp, flags, stream)
        if st == AMPH_E_PARAM and not _is_dev(keep[0]) and self._ff_value(bad) >= 0:
            raise ValueError(lib.amph_last_error().decode())
        self._check(st, allow_verify=True)
        return out, self._ff_value(ff), self._ff_value(bad)

    def mask_input_b64(self, texts, words: int, secrets16, records: bool = True, raw: bool = False):
        """amph_mask_input_b64: (masked (S, 16) or None, records (S, 24) or
        None, first_fail, bad_char)."""
        arr, keep = self._text_structs(texts)
        sv = words_view(secrets16)
        flags, stream = self._mode(sv, *keep)
        S = sv.shape[0]
        o16 = self._empty(sv, (S, 16)) if raw else None
        o24 = self._empty(sv, (S, 24)) if records else None
        ff, ffp = self._ff(sv)
        bad, badp = self._ff(sv)
        st = lib.amph_mask_input_b64(self._h, arr, len(texts), words, _ptr(sv), S,
                                     _ptr(o16) if raw else None, _ptr(o24) if records else None,
                                     ffp, badp, flags, stream)
        if st == AMPH_E_PARAM and not _is_dev(sv) and self._ff_value(bad) >= 0:
            raise ValueError(lib.amph_last_error().decode())
        self._check(st, allow_verify=True)
        return o16, o24, self._ff_value(ff), self._ff_value(bad)

    # -- wire codec (base64 as Jackson writes byte[]) ---------------------------
    def base64_encode(self, data) -> bytes:
        """bytes / uint8 array -> base64 ASCII (bytes); device tensor -> device tensor."""
        a = data if _is_dev(data) else np.frombuffer(bytes(data), np.uint8) \
            if isinstance(data, (bytes, bytearray, memoryview)) else np.ascontiguousarray(data, np.uint8).reshape(-1)
        n = a.numel() if _is_dev(a) else a.size
        flags, stream = self._mode(a)
        out = self._empty(a, (4 * ((n + 2) // 3),))
        self._check(lib.amph_base64_encode(self._h, _ptr(a), n, _ptr(out), flags, stream))
        return out if _is_dev(a) else out.tobytes()

    def base64_decode(self, text, nbytes: int | None = None) -> bytes:
        """base64 ASCII (str / bytes / uint8 array) -> bytes; raises ValueError on
        an illegal character or a length not divisible by 4.  Device text ->
        (uint8 tensor, bad-index word); with nbytes (the decoded length the
        caller expects, e.g. 16 per word of an ODO field) the call is fully
        asynchronous (no read-back of the padding to size the output).
        nbytes must then EQUAL the text's decoded length, 3 n / 4 minus its
        '=' padding: it is only range-checked here (the padding is on the
        device), and a wrong value returns a slice that cuts decoded bytes
        (too small) or ends in bytes the kernel never wrote (too large)."""
        if isinstance(text, str):
            text = text.encode("ascii", errors="replace")
        a = text if _is_dev(text) else np.frombuffer(bytes(text), np.uint8) \
            if isinstance(text, (bytes, bytearray, memoryview)) else np.ascontiguousarray(text, np.uint8).reshape(-1)
        n = a.numel() if _is_dev(a) else a.size
        flags, stream = self._mode(a)
        out = self._empty(a, (3 * n // 4,))
        ob = C.c_size_t(0)
        async_dev = _is_dev(a) and nbytes is not None
        if async_dev and not (n % 4 == 0 and 3 * n // 4 - 2 <= nbytes <= 3 * n // 4):
            raise ValueError("nbytes %d does not fit a %d-character text" % (nbytes, n))
        bad, badp = self._ff(a)
        st = lib.amph_base64_decode(self._h, _ptr(a), n, _ptr(out), None if async_dev else C.byref(ob), badp,
                                    flags, stream)
        if st in (AMPH_E_PARAM, AMPH_E_LEN):
            raise ValueError(lib.amph_last_error().decode())
        self._check(st)
        if _is_dev(a):
            return out[: nbytes if async_dev else ob.value], bad
        return out[: ob.value].tobytes()

    def base64_encode_words(self, words16):
        w = words_view(words16)
        flags, stream = self._mode(w)
        out = self._empty(w, (w.shape[0], 24))
        self._check(lib.amph_base64_encode_words(self._h, _ptr(w), w.shape[0], _ptr(out), flags, stream))
        return out

    def base64_decode_words(self, records24):
        r = words_view(records24, 24)
        flags, stream = self._mode(r)
        out = self._empty(r, (r.shape[0], 16))
        bad, badp = self._ff(r)
        st = lib.amph_base64_decode_words(self._h, _ptr(r), r.shape[0], _ptr(out), badp, flags, stream)
        if st == AMPH_E_PARAM and not _is_dev(r):
            raise ValueError(lib.amph_last_error().decode())
        self._check(st)
        return out if not _is_dev(r) else (out, bad)

    # -- Beaver open exchange (MultiplicationExchangeObject.interimValues) ------
    def exchange_encode(self, mag, neg):
        """Signed diffs (amph_odo_pre layout: mag (P, 2, 16), neg (P, 2)) -> the
        FactorPair JSON array text.  Host arrays -> bytes; device tensors ->
        (uint8 tensor with capacity amph_exchange_max_chars(P), length tensor)."""
        m = mag if _is_dev(mag) else np.ascontiguousarray(mag, np.uint8)
        g = neg if _is_dev(neg) else np.ascontiguousarray(neg, np.uint8)
        flags, stream = self._mode(m, g)
        P = m.shape[0]
        cap = lib.amph_exchange_max_chars(P)
        out = self._empty(m, (cap,))
        if _is_dev(m):
            import torch
            n = torch.empty(1, dtype=torch.int64, device=m.device)
            self._check(lib.amph_exchange_encode(self._h, _ptr(m), _ptr(g), P, _ptr(out), cap,
                                                 C.c_void_p(n.data_ptr()), flags, stream))
            return out, n
        n = C.c_uint64(0)
        self._check(lib.amph_exchange_encode(self._h, _ptr(m), _ptr(g), P, _ptr(out), cap,
                                             C.addressof(n), flags, stream))
        return out[: n.value].tobytes()

    def exchange_decode(self, text, npairs: int):
        """FactorPair JSON array text -> (mag (P, 2, 16), neg (P, 2)); raises
        ValueError on a malformed token or a count other than npairs.  Device
        uint8 tensor in -> (mag, neg, bad) device tensors, bad = AMPH_NO_FAILURE
        when clean."""
        if isinstance(text, str):
            text = text.encode("utf-8")
        a = text if _is_dev(text) else np.frombuffer(bytes(text), np.uint8)
        n = a.numel() if _is_dev(a) else a.size
        flags, stream = self._mode(a)
        mag = self._empty(a, (npairs, 2, 16))
        neg = self._empty(a, (npairs, 2))
        bad, badp = self._ff(a)
        st = lib.amph_exchange_decode(self._h, _ptr(a), n, npairs, _ptr(mag), _ptr(neg), badp, flags,
                                      stream)
        if st in (AMPH_E_PARAM, AMPH_E_LEN) and not _is_dev(a):
            raise ValueError(lib.amph_last_error().decode())
        self._check(st)
        return (mag, neg) if not _is_dev(a) else (mag, neg, bad)

    # -- one party's Output Delivery, device-resident between steps ------------
    def party_begin(self, share_data, share_stride: int, masks32, triples96, n_parties: int,
                    want_yrv: bool = True) -> "PartySession":
        """amph_party_begin from host buffers: the tuples in, (y, r, v) out
        (unless want_yrv is False), this party's interimValues text kept on
        the device (PartySession.text())."""
        sd = words_view(share_data, share_stride)
        mk, tr = words_view(masks32, 32), words_view(triples96, 96)
        W = sd.shape[0]
        _need(mk.shape[0] == 2 * W, "expected %d input-mask tuples, got %d" % (2 * W, mk.shape[0]))
        _need(tr.shape[0] == 2 * W, "expected %d multiplication triples, got %d" % (2 * W, tr.shape[0]))
        yrv = tuple(np.empty((W, 16), np.uint8) for _ in range(3)) if want_yrv else (None, None, None)
        h = C.c_void_p()
        self._check(lib.amph_party_begin(self._h, _ptr(sd), share_stride, _ptr(mk), _ptr(tr), W, n_parties,
                                         *[_ptr(x) for x in yrv], C.byref(h)))
        return PartySession(self, h, W, n_parties, yrv)

    def party_begin_dev(self, share_data, share_stride: int, masks32, triples96, n_parties: int,
                        want_yrv: bool = False) -> "PartySessionDev":
        """amph_party_begin_dev on torch device tensors (used in place; the
        triples must stay unchanged until finish), asynchronous on torch's
        current stream."""
        import torch
        W = share_data.shape[0]
        _need(share_data.is_cuda and masks32.is_cuda and triples96.is_cuda, "device tensors expected")
        _need(share_data.numel() == W * share_stride, "share data: %d words of %d bytes" % (W, share_stride))
        _need(masks32.numel() == 64 * W, "expected %d input-mask tuples" % (2 * W))
        _need(triples96.numel() == 192 * W, "expected %d multiplication triples" % (2 * W))
        yrv = tuple(torch.empty((W, 16), dtype=torch.uint8, device=share_data.device) for _ in range(3)) \
            if want_yrv else (None, None, None)
        stream = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        h = C.c_void_p()
        self._check(lib.amph_party_begin_dev(self._h, _ptr(share_data), share_stride, _ptr(masks32),
                                             _ptr(triples96), W, n_parties, *[_ptr(x) for x in yrv], stream,
                                             C.byref(h)))
        return PartySessionDev(self, h, W, n_parties, yrv, (share_data, masks32, triples96))

    # -- synthetic device inputs (bench / tests) --------------------------------
    def synth_odos(self, seed: int, n: int, words: int, fault_index: int = -1,
                   noncanon_permille: int = 0, with_plain: bool = False, buf=None):
        """Returns (odos, buffer, plain_y): a (5, n, W, 16) uint8 device
        tensor, the per-party (y, r, v, w, u) views of it, optional secrets.
        `buf`: generate into the caller's (5, n, W, 16) device tensor."""
        import torch
        if buf is None:
            buf = torch.empty((5, n, words, 16), dtype=torch.uint8, device="cuda:%d" % self.device)
        elif (tuple(buf.shape[:2]) != (5, n) or buf.shape[2] < words or tuple(buf.shape[3:]) != (16,)
              or buf.dtype != torch.uint8 or not buf.is_contiguous()):
            raise ValueError("buf must be a contiguous (5, n, >= words, 16) uint8 device tensor")
        buf = buf[:, :, :words]  # a padded slab: each field starts at its own row of the slab
        plain = torch.empty((words, 16), dtype=torch.uint8, device=buf.device) if with_plain else None
        ptrs = (C.c_void_p * (5 * n))(*[buf[k, j].data_ptr() for k in range(5) for j in range(n)])
        stream = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        self._check(lib.amph_synth_odos(self._h, seed, n, words, ptrs, _ptr(plain), fault_index,
                                        noncanon_permille, stream))
        odos = [tuple(buf[k, j] for k in range(5)) for j in range(n)]
        return odos, buf, plain

    def synth_words(self, seed: int, count: int, out=None):
        import torch
        if out is None:
            out = torch.empty((count, 16), dtype=torch.uint8, device="cuda:%d" % self.device)
        elif tuple(out.shape) != (count, 16) or out.dtype != torch.uint8 or not out.is_contiguous():
            raise ValueError("out must be a contiguous (count, 16) uint8 device tensor")
        stream = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        self._check(lib.amph_synth_words(self._h, seed, count, _ptr(out), stream))
        return out


class PartySession:
    """One amph_party (include/amphora.h): a party's Output Delivery with the
    triples, diffs and ODO fields kept on the device between begin, the
    partners' texts and finish."""

    def __init__(self, ctx: Context, h, words: int, n_parties: int, yrv):
        self.ctx, self._h, self.words, self.n = ctx, h, words, n_parties
        self.y, self.r, self.v = yrv

    def text(self) -> bytes:
        """This party's interimValues text (the FactorPair JSON array)."""
        n = lib.amph_party_text_len(self._h)
        out = np.empty(max(n, 1), np.uint8)
        Context._check(lib.amph_party_text(self._h, _ptr(out), n))
        return out[:n].tobytes()

    def partner(self, slot: int, text):
        """A partner's interimValues text into slot 1..n-1; raises ValueError
        on a malformed text or a pair count other than 2 * words."""
        if isinstance(text, str):
            text = text.encode("utf-8")
        a = np.frombuffer(bytes(text), np.uint8)
        bad = C.c_int64(-1)
        st = lib.amph_party_partner(self._h, slot, _ptr(a) if a.size else None, a.size, C.byref(bad))
        if st in (AMPH_E_PARAM, AMPH_E_LEN) and bad.value >= 0:
            raise ValueError(lib.amph_last_error().decode())
        Context._check(st)

    def finish(self, is_player0: bool):
        """-> (w, u) as (W, 16) words."""
        w, u = np.empty((self.words, 16), np.uint8), np.empty((self.words, 16), np.uint8)
        Context._check(lib.amph_party_finish(self._h, int(is_player0), _ptr(w), _ptr(u)))
        return w, u

    def finish_b64(self, is_player0: bool):
        """-> the five ODO fields (secretShares, rShares, vShares, wShares,
        uShares) as base64 bytes."""
        nc = 4 * ((16 * self.words + 2) // 3)
        outs = [np.empty(max(nc, 1), np.uint8) for _ in range(5)]
        arr = (C.c_void_p * 5)(*[_ptr(o) for o in outs])
        Context._check(lib.amph_party_finish_b64(self._h, int(is_player0), arr))
        return [o[:nc].tobytes() for o in outs]

    def reset_partner(self, slot: int):
        """amph_party_reset_partner: free a slot whose text was rejected."""
        Context._check(lib.amph_party_reset_partner(self._h, slot))

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            lib.amph_party_free(self._h)
        self._h = None

    def __del__(self):
        if lib is not None:
            self.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class _DevArray:  # a device address as __cuda_array_interface__ (torch.as_tensor views it)
    def __init__(self, ptr: int, n: int, typestr: str):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (ptr, False), "version": 2}


def _dev_view(ptr: int, n: int, typestr: str, device: int):
    import torch
    return torch.as_tensor(_DevArray(ptr, n, typestr), device="cuda:%d" % device)


class PartySessionDev(PartySession):
    """A device-mode amph_party (amph_party_*_dev): torch device tensors in
    and out, every call asynchronous on torch's current stream."""

    def __init__(self, ctx: Context, h, words: int, n_parties: int, yrv, keep):
        super().__init__(ctx, h, words, n_parties, yrv)
        self._keep = keep  # the tuples, read in place until finish

    def _stream(self):
        import torch
        return C.c_void_p(torch.cuda.current_stream(self.ctx.device).cuda_stream)

    def text_dev(self):
        """-> (this party's text: a uint8 device tensor of the text's capacity,
        its length: an int64 (1,) device tensor), both views of session memory
        (amph_party_text_dev), valid once the stream has run begin."""
        t, n = C.c_void_p(), C.c_void_p()
        Context._check(lib.amph_party_text_dev(self._h, C.byref(t), C.byref(n)))
        cap = lib.amph_exchange_max_chars(2 * self.words)
        return _dev_view(t.value, cap, "|u1", self.ctx.device), _dev_view(n.value, 1, "<i8", self.ctx.device)

    def text(self) -> bytes:
        """Synchronises and copies this party's text to the host (tests)."""
        t, n = self.text_dev()
        L = int(n.item())
        return t[:L].cpu().numpy().tobytes()

    def partner(self, slot: int, text, bad=None):
        """A partner's text (a uint8 device tensor) into slot 1..n-1; bad: an
        int64 (1,) device tensor the decode reports into (returned)."""
        import torch
        if bad is None:
            bad = torch.empty(1, dtype=torch.int64, device=text.device)
        Context._check(lib.amph_party_partner_dev(self._h, slot, _ptr(text) if text.numel() else None,
                                                  text.numel(), _ptr(bad), self._stream()))
        return bad

    def finish(self, is_player0: bool):
        raise AmphoraNativeError(AMPH_E_PARAM, "a device-mode session finishes with finish_b64")

    def finish_b64(self, is_player0: bool):
        """-> the five fields' base64 text: uint8 device tensors viewing the
        session's memory (valid until close)."""
        nc = 4 * ((16 * self.words + 2) // 3)
        arr = (C.c_void_p * 5)()
        Context._check(lib.amph_party_finish_b64_dev(self._h, int(is_player0), arr, self._stream()))
        return [_dev_view(arr[k], nc, "|u1", self.ctx.device) if nc else None for k in range(5)]

