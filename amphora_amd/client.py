"""Host-side mirror of the client arithmetic (amphora-java-client), routed to
the HIP kernels through the C ABI.

Mirrors:
* SecretShareUtil            amphora-java-client/.../client/SecretShareUtil.java:33-157
  (of :48-51, maskInput :65-68, recombineObject :70-90, verifySecrets :102-141)
* DefaultAmphoraClient.verifyOutputDeliveryObjects :476-505 and the
  arithmetic of createSecret :150-160 / getSecret :206-217.

Java BigIntegers are Python ints here.  Host-side obligations of the
boundary: arbitrary ints are reduced mod p before packing into
16-byte words; canonical outputs are unpacked back to ints.  No field
arithmetic happens in Python.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np

from . import _lib
from .entities import (AmphoraClientException, IntegrityVerificationException, MaskedInput,
                       MaskedInputData, MaskedInputWords, OutputDeliveryObject, Secret, WORD_WIDTH)

_MASK128 = (1 << 128) - 1


def pack(values: Sequence[int], prime: int = None) -> np.ndarray:
    """ints -> (W, 16) LE words; reduced mod prime when given (BigInteger.mod)."""
    if prime is not None:
        values = [v % prime if (v < 0 or v > _MASK128) else v for v in values]
    buf = b"".join(int(v).to_bytes(16, "little") for v in values)
    return np.frombuffer(buf, np.uint8).reshape(-1, 16).copy() if buf else np.zeros((0, 16), np.uint8)


def unpack(words) -> List[int]:
    if hasattr(words, "is_cuda"):
        words = words.cpu().numpy()
    b = np.ascontiguousarray(words, np.uint8).tobytes()
    return [int.from_bytes(b[i:i + 16], "little") for i in range(0, len(b), 16)]


class SecretShareUtil:
    """Client SecretShareUtil; ``of`` keeps the reference factory signature."""

    def __init__(self, ctx: _lib.Context):
        self._ctx = ctx

    @classmethod
    def of(cls, prime: int, r: int, r_inv: int, device: int = 0) -> "SecretShareUtil":
        if prime is None or r is None or r_inv is None:
            raise TypeError("prime, r and rInv must not be null")  # @NonNull :48-49
        return cls(_lib.Context(prime, r, r_inv, device))

    @property
    def prime(self) -> int:
        return self._ctx.prime

    @property
    def r(self) -> int:
        return self._ctx.r

    @property
    def r_inv(self) -> int:
        return self._ctx.r_inv

    @property
    def context(self) -> _lib.Context:
        return self._ctx

    def mask_input(self, secret: int, input_mask: int) -> MaskedInputData:
        """maskInput :65-68: MaskedInputData.of(toGfp((secret - inputMask) mod p))."""
        return self.mask_inputs([secret], [input_mask])[0]

    def mask_inputs(self, secrets: Sequence[int], input_masks: Sequence[int]) -> List[MaskedInputData]:
        out = self._ctx.mask_words(pack(secrets, self.prime), pack(input_masks, self.prime))
        return [MaskedInputData.of(bytes(w)) for w in out]

    def recombine_object(self, shares: Sequence[bytes]) -> List[int]:
        """recombineObject :70-90 (word count from shares[0], trailing bytes ignored)."""
        if len(shares) == 0:
            return []
        W = len(shares[0]) // WORD_WIDTH
        views = [_lib.words_view(s)[:W] for s in shares]
        if any(v.shape[0] < W for v in views):
            raise IndexError("share arrays shorter than the first")
        return unpack(self._ctx.recombine(views))

    def verify_secrets(self, secrets, rs, us, vs, ws) -> None:
        """verifySecrets :102-141 (argument order of the Java method)."""
        n = len(secrets)
        p = self.prime
        # host precheck: a w/u outside [0, p) can never equal a reduced product
        pre = [i for i in range(n) if not (0 <= ws[i] < p and 0 <= us[i] < p)]
        ok_w = [w if 0 <= w < p else 0 for w in ws]
        ok_u = [u if 0 <= u < p else 0 for u in us]
        ff = self._ctx.verify(pack(secrets, p), pack(rs, p), pack(ok_u), pack(vs, p), pack(ok_w))
        cand = [i for i in ([ff] if ff >= 0 else []) + pre[:1]]
        if cand:
            i = min(cand)
            raise IntegrityVerificationException(
                self.failure_message(secrets[i], rs[i], us[i], vs[i], ws[i]))

    def failure_message(self, y, r, u, v, w) -> str:
        """Message of SecretShareUtil.java:116-129; products computed natively."""
        p = self.prime
        fits = all(0 <= x <= _MASK128 for x in (y, r, u, v, w))
        if fits:
            return self._ctx.verify_message(y, r, u, v, w)
        msg = self._ctx.verify_message(y % p, r % p, u % p, v % p, w % p)
        tail = msg.split("\n")[-1]  # "\t{w} = {aw}   &&   {u} = {au}"
        aw = tail.split("   &&   ")[0].split(" = ")[1]
        au = tail.split("   &&   ")[1].split(" = ")[1]
        return ("Verification of secret has failed:\n\t%d = %d * %d   &&   %d = %d * %d\n"
                "\t%d = %s   &&   %d = %s" % (w, y, r, u, v, r, w, aw, u, au))


def _odo_arrays(odos: Sequence[OutputDeliveryObject]):
    """Every party's five fields as they are, with their own byte lengths:
    the C ABI applies recombineObject's copyOfRange rules to ragged parties
    (client SecretShareUtil.java:75,87-88), so nothing is cut here."""
    return [tuple(o.fields()) for o in odos]


def _words(arrays) -> int:
    return _lib.byte_len(arrays[0][0]) // WORD_WIDTH  # party 0's word count (:75)


def verify_output_delivery_objects(util: SecretShareUtil,
                                   odos: Sequence[OutputDeliveryObject]) -> List[int]:
    """DefaultAmphoraClient.verifyOutputDeliveryObjects :476-505, fused into one
    kernel (K_RV): 5 recombines + verify, returns the canonical secrets."""
    arrays = _odo_arrays(odos)
    y, ff = _native(util.context.recombine_verify, arrays)
    if ff >= 0:
        _raise_for(util, arrays, ff)
    return unpack(y)


def _native(fn, *args):
    """A C-ABI call whose AMPH_E_RANGE (a party's word starting past the end
    of its array) is Java's ArrayIndexOutOfBoundsException (IndexError)."""
    try:
        return fn(*args)
    except _lib.AmphoraNativeError as e:
        if e.status == _lib.AMPH_E_RANGE:
            raise IndexError(str(e)) from e
        raise


def _raise_for(util: SecretShareUtil, arrays, i: int):
    """Re-render the reference message for word i from its recombined values:
    each party's word i is Arrays.copyOfRange(field, 16 i, 16 i + 16) --
    zero-padded when the party's array ends inside it -- exactly what
    recombineObject hands fromGfp (amph_recombine_object on those slices)."""
    lo, hi = WORD_WIDTH * i, WORD_WIDTH * (i + 1)
    vals = [unpack(util.context.recombine_object([_slice(a[k], lo, hi) for a in arrays]))[0]
            for k in range(5)]
    y, r, v, w, u = vals
    raise IntegrityVerificationException(util.failure_message(y, r, u, v, w))


def _slice(x, lo: int, hi: int):
    if hasattr(x, "is_cuda"):
        return x.reshape(-1)[lo:hi]
    return bytes(memoryview(x).cast("B")[lo:hi]) if not isinstance(x, bytes) else x[lo:hi]


def create_masked_input(util: SecretShareUtil, secret: Secret,
                        mask_odos: Sequence[OutputDeliveryObject]) -> MaskedInput:
    """Arithmetic of DefaultAmphoraClient.createSecret :150-160 fused into one
    kernel (K_MASK): verify the Input Mask ODOs, then maskInput per word.
    More secret words than masks: the C ABI verifies every mask first
    (:153) and only then reports the length (AMPH_E_LEN), which is the
    reference's IndexOutOfBoundsException from inputMasks.get(i) (:155-157)."""
    arrays = _odo_arrays(mask_odos)
    W = _words(arrays)
    try:
        masked, ff = _native(util.context.mask_input, arrays, pack(secret.data, util.prime))
    except _lib.AmphoraNativeError as e:
        if e.status == _lib.AMPH_E_LEN and secret.size() > W:
            raise IndexError("Index %d out of bounds for length %d" % (W, W)) from e
        raise
    if ff >= 0:
        _raise_for(util, arrays, ff)
    return MaskedInput(secret.secret_id, MaskedInputWords(masked), list(secret.tags))


def _texts_and_words(bodies):
    """Field texts of every party's body and the word count.  A malformed
    body -- a field that is not a whole number of 16-byte words, or fields of
    unequal length within or across parties -- is an AmphoraClientException,
    as Jackson's deserialisation failure is in the reference
    (DefaultAmphoraClient.java:206-217 via AmphoraCommunicationClient)."""
    from . import wire
    texts = [wire.odo_field_texts(b)[0] for b in bodies]
    try:
        W = wire.words_of_b64(len(texts[0][0]), texts[0][0][-2:])
    except ValueError as e:
        raise AmphoraClientException(str(e)) from e
    n0 = len(texts[0][0])
    if any(len(f) != n0 for t in texts for f in t):
        # OutputDeliveryObject's constructor (OutputDeliveryObject.java:55-96)
        raise AmphoraClientException("The provided shares must be of the same length")
    return texts, W


def _wire_call(fn, *args, **kw):
    """A fused wire-kernel call; a bad character or a length mismatch in some
    party's text becomes AmphoraClientException."""
    try:
        return fn(*args, **kw)
    except ValueError as e:  # an illegal base64 character in some party's body
        raise AmphoraClientException(str(e)) from e
    except _lib.AmphoraNativeError as e:
        if e.status == _lib.AMPH_E_LEN:
            raise AmphoraClientException(str(e)) from e
        raise


def _raise_for_texts(util: SecretShareUtil, texts, i: int):
    # failure path only: decode the fields and render the reference message
    arrays = [tuple(util.context.base64_decode(t) for t in ts) for ts in texts]
    _raise_for(util, arrays, i)


def verify_vss_json(util: SecretShareUtil, bodies: Sequence[str], secret_id=None):
    """getSecret from the parties' VerifiableSecretShare JSON bodies
    (DefaultAmphoraClient.java:206-217 incl. Jackson's base64 decode of each
    field): the base64 member strings go to the fused K_RV wire kernel
    (amph_recombine_verify_b64) as they are.  Returns (secretId, tags,
    canonical secrets).  As in the reference (:213-216) the secretId is the
    one requested (`secret_id`; party 0's body only when none is given) and
    only the tags come from party 0's body."""
    from . import wire
    texts, W = _texts_and_words(bodies)
    y, ff, _ = _wire_call(util.context.recombine_verify_b64, texts, W)
    if ff >= 0:
        _raise_for_texts(util, texts, ff)
    sid, tags = wire.vss_metadata(bodies[0], wire.odo_field_texts(bodies[0])[1])
    return (sid if secret_id is None else secret_id), tags, unpack(y)


def create_masked_input_json(util: SecretShareUtil, secret: Secret, odo_bodies: Sequence[str]) -> str:
    """createSecret from the parties' OutputDeliveryObject JSON bodies
    (GET /input-masks) to the MaskedInput JSON body (POST /masked-inputs):
    verify the masks + maskInput + the per-word base64 records in one fused
    launch (amph_mask_input_b64)."""
    from . import wire
    texts, W = _texts_and_words(odo_bodies)
    try:
        # more secret words than masks: the ABI decodes and verifies every
        # mask first (a MAC failure comes back as ff), and only then reports
        # the length -- the reference's order (:153 before :155-157)
        _, rec, ff, _ = _wire_call(util.context.mask_input_b64, texts, W, pack(secret.data, util.prime),
                                   records=True)
    except AmphoraClientException as e:
        if secret.size() > W and isinstance(e.__cause__, _lib.AmphoraNativeError) \
                and e.__cause__.status == _lib.AMPH_E_LEN:
            raise IndexError("Index %d out of bounds for length %d" % (W, W)) from e.__cause__
        raise
    if ff >= 0:
        _raise_for_texts(util, texts, ff)
    return wire.records_to_masked_input_json(secret.secret_id, rec, secret.tags)


def get_secret_data(util: SecretShareUtil, odos: Sequence[OutputDeliveryObject]) -> List[int]:
    """getSecret :206-217 arithmetic (alias of verify_output_delivery_objects)."""
    return verify_output_delivery_objects(util, odos)
