"""CPU-only checks of the C ABI: the library loads, exports every function
include/amphora.h declares, validates field parameters, and renders the
reference's verification message (host-side code, no GPU needed)."""
import ctypes
import os
import re

import pytest

from oracle import amphora_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P, R, RINV = O.TEST_PRIME, O.TEST_R, O.TEST_RINV


def header_functions():
    src = open(os.path.join(ROOT, "include", "amphora.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(amph_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_header(native):
    lib = ctypes.CDLL(native._lib.LIB_PATH)
    names = header_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), n
    assert sorted(native._lib.EXPORTED) == names


@pytest.fixture(scope="module")
def native():
    import amphora_amd
    return amphora_amd


def test_ctx_param_validation(native):
    native.Context(P, R, RINV)
    with pytest.raises(native.AmphoraNativeError, match="r must equal"):
        native.Context(P, R + 1, RINV)
    with pytest.raises(native.AmphoraNativeError, match="inverse"):
        native.Context(P, R, RINV + 1)
    with pytest.raises(native.AmphoraNativeError, match="odd"):
        native.Context(P + 1, R, RINV)


def test_verify_message_matches_reference_format(native):
    c = native.Context(P, R, RINV)
    util = O.ClientSecretShareUtil(P, R, RINV)
    s, r, v = 123456789, 987654321, 55555
    w, u = s * r - 10, v * r
    expected = O.verification_failure_message(P, 0, [s], [r], [u], [v], [w])
    assert c.verify_message(s, r, u, v, w) == expected
    big = [P - 1, P - 2, P - 3]
    exp = O.verification_failure_message(P, 0, [big[0]], [big[1]], [5], [big[2]], [7])
    assert c.verify_message(big[0], big[1], 5, big[2], 7) == exp
    assert util  # oracle and native render the same text


def test_entities_invariants(native):
    from amphora_amd import entities as E
    with pytest.raises(E.IllegalArgumentException, match="same length"):
        E.OutputDeliveryObject(b"\0" * 16, b"\0" * 16, b"\0" * 32, b"\0" * 16, b"\0" * 16)
    with pytest.raises(E.IllegalArgumentException, match="has to be 16 bytes"):
        E.MaskedInputData.of(b"\0" * 15)
    with pytest.raises(E.IllegalArgumentException, match="multiple of 32"):
        E.SecretShare(None, b"\0" * 48)
    # MaskedInputTest.java: null id rejected, null tags -> empty list
    with pytest.raises(E.NullPointerException, match="^secretId is marked non-null but is null$"):
        E.MaskedInput(None, [], [])
    import uuid
    sid = uuid.UUID("80fbba1b-3da8-4b1e-8a2c-cebd65229fad")
    mi = E.MaskedInput(sid, [E.MaskedInputData.of(bytes(16))], None)
    assert mi.secret_id == sid and mi.tags == []
    with pytest.raises(E.IllegalArgumentException, match="^Length of a Masked Input value has to be 16 bytes.$"):
        E.MaskedInputData.of(bytes(15))


def test_name_uuid(native):
    from amphora_amd.service import name_uuid_from_bytes
    assert str(name_uuid_from_bytes(b"70297fd4-d412-4dbb-af05-6818fe0e687a_4")) == \
        "8065e700-9f48-36ba-ae8c-f881b28a28ef"


def test_no_gpu_fails_loudly(native):
    import numpy as np
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    c = native.Context(P, R, RINV)
    with pytest.raises(native.AmphoraNativeError, match="HIP"):
        c.recombine_verify([(np.zeros((4, 16), np.uint8),) * 5])


def test_param_validation_before_any_device_work(native):
    """Argument checks return AMPH_E_PARAM / AMPH_E_LEN with a message before
    the library touches a device (runs without a GPU)."""
    L = native._lib.lib
    c = native.Context(P, R, RINV)
    ff = ctypes.c_int64(0)
    assert L.amph_recombine_verify(c._h, None, 0, None, ctypes.byref(ff), 0, None) == native._lib.AMPH_E_PARAM
    assert b"n_parties" in L.amph_last_error()
    assert L.amph_recombine_verify(c._h, None, 17, None, ctypes.byref(ff), 0, None) == native._lib.AMPH_E_PARAM
    n = ctypes.c_uint64(0)
    assert L.amph_exchange_encode(c._h, None, None, 5, None, 0, ctypes.addressof(n), 0, None) == \
        native._lib.AMPH_E_PARAM
    assert L.amph_exchange_decode(c._h, None, 4, 0, None, None, None, 0, None) == native._lib.AMPH_E_PARAM
    assert L.amph_base64_decode(c._h, b"abc", 3, None, None, None, 0, None) in (
        native._lib.AMPH_E_LEN, native._lib.AMPH_E_PARAM)
    # {"a":-<39>,"b":-<39>}, = 92 chars per pair + the brackets
    assert L.amph_exchange_max_chars(10) == 922
    assert L.amph_exchange_max_chars(0) == 2
    for code in range(6):
        assert L.amph_strerror(code)


def test_multi_device_context_validation(native):
    """amph_ctx_create_multi: argument checks and device count (no GPU work)."""
    L = native._lib.lib
    h = ctypes.c_void_p()
    keys = [native._lib.le16(x) for x in (P, R, RINV)]
    assert L.amph_ctx_create_multi(*keys, None, 2, ctypes.byref(h)) == native._lib.AMPH_E_PARAM
    devs = (ctypes.c_int * 3)(0, 0, 0)
    assert L.amph_ctx_create_multi(*keys, devs, 0, ctypes.byref(h)) == native._lib.AMPH_E_PARAM
    c = native.Context(P, R, RINV, devices=[0, 0, 0])
    assert c.device_count == 3 and c.device == 0
    assert native.Context(P, R, RINV, devices=[0]).device_count == 1
    with pytest.raises(native.AmphoraNativeError, match="inverse"):
        native.Context(P, R, RINV + 1, devices=[0, 0])


def test_out_buffer_validation(native):
    """out= must be a C-contiguous uint8 buffer of the output's exact shape,
    in the same memory as the inputs (checked before any device work)."""
    import numpy as np
    c = native.Context(P, R, RINV)
    odo = [(np.zeros((4, 16), np.uint8),) * 5]
    for bad in (np.zeros((3, 16), np.uint8), np.zeros((4, 16), np.int32),
                np.zeros((16, 4), np.uint8).T):
        with pytest.raises(ValueError, match="out must be"):
            c.recombine_verify(odo, out=bad)
        with pytest.raises(ValueError, match="out must be"):
            c.mask_input(odo, np.zeros((4, 16), np.uint8), out=bad)


def test_byte_len_is_the_length_of_what_c_reads(native):
    """byte_len and words_view agree for every host input form:
    the length handed to C is the length of the uint8 buffer whose pointer is
    passed, so an int64 array or a list is never reported at 8x its size."""
    import numpy as np
    from amphora_amd._lib import byte_len, words_view
    for x in (np.arange(40, dtype=np.int64), list(range(40)), bytes(40), bytearray(40),
              np.zeros(40, np.uint8), memoryview(bytes(40)), np.zeros((5, 8), np.uint16)):
        v = words_view(x)
        assert byte_len(x) == 40, type(x)
        assert v.nbytes == 32 and v.shape == (2, 16)  # whole words of the same buffer
