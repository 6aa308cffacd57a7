"""CPU oracle for Amphora's per-word secret-share arithmetic.

TEST INFRASTRUCTURE ONLY.  Nothing in the product path (``amphora_amd``,
``libamphora_hip.so``) may import, call or link this module.  Only ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` use it,
and only as the checker.

This is a pure-Python-``int`` restatement of the Java ``BigInteger`` code of
carbynestack/amphora (reference snapshot 2025-03-21).  Every function cites
the reference ``file:line`` it follows.  Python ``int`` has the same
arbitrary-precision semantics as ``java.math.BigInteger`` for ``add``,
``subtract``, ``multiply`` and ``mod`` (``BigInteger.mod`` always returns a
value in ``[0, m)``; so does Python's ``%`` for a positive modulus).

Third-party arithmetic restated here (absent from /root/reference):

* ``io.carbynestack:mp-spdz-integration:0.2.2``
  (``amphora-parent/pom.xml:60,167-169``) -- ``MpSpdzIntegrationUtils``:
  ``toGfp(x) = LE16((x * R) mod p)``, ``fromGfp(b) = (LEint(b) * R^-1) mod p``,
  ``WORD_WIDTH = 16``, ``SHARE_WIDTH = 32``.  The *value-level* behaviour is
  pinned by the reference's own known-answer tests (KAT-1, KAT-2 below); the
  *byte order* (little-endian Montgomery limbs, MP-SPDZ's native gfp layout)
  is the documented assumption ``ENCODING = "mont_le"``: the
  reference's tests compose toGfp/fromGfp symmetrically, so any bijective
  encoding passes them.
* ``io.carbynestack:castor-common:0.2.0`` (``amphora-parent/pom.xml:58,157-159``)
  -- tuple byte layouts only: an InputMask tuple is one share
  ``value(16) || mac(16)``; a MultiplicationTriple is three shares
  ``a||mac_a||b||mac_b||c||mac_c`` (96 B), as built by hand in
  ``OutputDeliveryServiceTest.java:80-154``.

Pins: ``tests/test_oracle_kat.py`` checks this module against KAT-1
(``amphora-service/.../calculation/SecretShareUtilTest.java:68-107``), KAT-2
(``OutputDeliveryServiceTest.java:55-175,285-382``), the verify pass/fail
structure of ``amphora-java-client/.../SecretShareUtilTest.java:30-85`` and
the round-trip properties of ``DefaultAmphoraClientTest.java:193-271``.
"""
from __future__ import annotations

import hashlib
import uuid
from typing import List, Sequence, Tuple

ENCODING = "mont_le"

WORD_WIDTH = 16  # MpSpdzIntegrationUtils.WORD_WIDTH
SHARE_WIDTH = 32  # MpSpdzIntegrationUtils.SHARE_WIDTH
INPUT_MASK_TUPLE_SIZE = 32  # castor TupleType.INPUT_MASK_GFP.getTupleSize()
TRIPLE_TUPLE_SIZE = 96  # castor TupleType.MULTIPLICATION_TRIPLE_GFP.getTupleSize()

# Field used by every reference test (SecretShareUtilTest.java:24-28,
# application-test.properties:36-38).
TEST_PRIME = 198766463529478683931867765928436695041
TEST_R = 141515903391459779531506841503331516415
TEST_RINV = 133854242216446749056083838363708373830


class IntegrityVerificationException(Exception):
    """amphora-common/.../exceptions/IntegrityVerificationException.java:15-26"""


class IllegalArgumentException(ValueError):
    """java.lang.IllegalArgumentException as thrown on the path."""


class ArrayIndexOutOfBoundsException(IndexError):
    """java.lang.ArrayIndexOutOfBoundsException (Arrays.copyOfRange -> System.arraycopy)."""


def copy_of_range(original: bytes, frm: int, to: int) -> bytes:
    """java.util.Arrays.copyOfRange(byte[], from, to) (JDK 8-21): a new array
    of to - from bytes holding original[from:min(len, to)] and zeros after
    it; from > original.length throws ArrayIndexOutOfBoundsException (from ==
    length is allowed and gives all zeros), from > to IllegalArgumentException.
    recombineObject cuts every party's word with it (client
    SecretShareUtil.java:87-88), which is what gives ragged party arrays
    their meaning."""
    if frm > to:
        raise IllegalArgumentException("%d > %d" % (frm, to))
    if frm < 0 or frm > len(original):
        raise ArrayIndexOutOfBoundsException(
            "arraycopy: source index %d out of bounds for byte[%d]" % (frm, len(original)))
    part = bytes(original[frm:min(len(original), to)])
    return part + bytes(to - frm - len(part))


class MpSpdzIntegrationUtils:
    """Restatement of mp-spdz-integration 0.2.2 ``MpSpdzIntegrationUtils``.

    Call sites: client ``SecretShareUtil.java:50,56,67``; service
    ``SecretShareUtil.java:44,87-93,100``; ``OutputDeliveryService.java:129-131,
    150-151,194,199,278-280``.
    """

    WORD_WIDTH = WORD_WIDTH
    SHARE_WIDTH = SHARE_WIDTH

    def __init__(self, prime: int, r: int, r_inv: int):
        self.prime = prime
        self.r = r
        self.r_inv = r_inv

    @classmethod
    def of(cls, prime: int, r: int, r_inv: int) -> "MpSpdzIntegrationUtils":
        return cls(prime, r, r_inv)

    def to_gfp(self, value: int) -> bytes:
        """toGfp: BigInteger -> 16-byte Montgomery little-endian word."""
        return ((value * self.r) % self.prime).to_bytes(WORD_WIDTH, "little")

    def from_gfp(self, word: bytes) -> int:
        """fromGfp: 16-byte word -> canonical BigInteger in [0, p)."""
        if len(word) != WORD_WIDTH:
            raise IllegalArgumentException("word must be %d bytes" % WORD_WIDTH)
        return (int.from_bytes(word, "little") * self.r_inv) % self.prime


def words(buf: bytes) -> List[bytes]:
    """Split a byte[] into WORD_WIDTH words; a trailing partial word is
    dropped exactly as ``length / WORD_WIDTH`` does in Java."""
    n = len(buf) // WORD_WIDTH
    return [buf[i * WORD_WIDTH:(i + 1) * WORD_WIDTH] for i in range(n)]


# --------------------------------------------------------------------------
# Client side: amphora-java-client/.../client/SecretShareUtil.java
# --------------------------------------------------------------------------
class ClientSecretShareUtil:
    """amphora-java-client/src/main/java/io/carbynestack/amphora/client/SecretShareUtil.java"""

    def __init__(self, prime: int, r: int, r_inv: int):
        # SecretShareUtil.of  :48-51
        self.prime, self.r, self.r_inv = prime, r, r_inv
        self.spdz = MpSpdzIntegrationUtils.of(prime, r, r_inv)

    of = classmethod(lambda cls, prime, r, r_inv: cls(prime, r, r_inv))

    def mask_input(self, secret: int, input_mask: int) -> bytes:
        """maskInput :65-68 -> MaskedInputData.of(toGfp((s - m) mod p))."""
        return self.spdz.to_gfp((secret - input_mask) % self.prime)

    def recombine_object(self, shares: Sequence[bytes]) -> List[int]:
        """recombineObject :70-90 with summingGfpAsBigInteger :53-63.

        The word count comes from ``shares.get(0).length / WORD_WIDTH`` (:75);
        each party's word i is ``Arrays.copyOfRange(share, 16 i, 16 i + 16)``
        (:87-88), so parties of other lengths than party 0 are cut, or
        zero-padded past their end, or raise ArrayIndexOutOfBoundsException
        for a word that starts past their end (``copy_of_range``); each word
        is the BigInteger sum of fromGfp over parties, then mod p."""
        if len(shares) == 0:
            return []
        n_words = len(shares[0]) // WORD_WIDTH
        out = []
        for i in range(n_words):
            acc = 0
            for s in shares:
                acc += self.spdz.from_gfp(copy_of_range(s, i * WORD_WIDTH, (i + 1) * WORD_WIDTH))
            out.append(acc % self.prime)
        return out

    def verify_secrets(self, secrets, rs, us, vs, ws) -> None:
        """verifySecrets :102-141.  The Java loop is a parallel forEach and
        throws for *some* failing index; this restatement walks in index order
        and reports the smallest one (the deterministic choice the HIP path
        makes too).  Message format :116-129, ``%n`` = ``\\n`` on Linux."""
        idx = first_failing_index(self.prime, secrets, rs, us, vs, ws)
        if idx >= 0:
            raise IntegrityVerificationException(
                verification_failure_message(self.prime, idx, secrets, rs, us, vs, ws))


def first_failing_index(prime, secrets, rs, us, vs, ws) -> int:
    for i in range(len(secrets)):
        actual_w = (secrets[i] * rs[i]) % prime
        actual_u = (vs[i] * rs[i]) % prime
        if ws[i] != actual_w or us[i] != actual_u:
            return i
    return -1


def verification_failure_message(prime, i, secrets, rs, us, vs, ws) -> str:
    """String.format of SecretShareUtil.java:116-129 for index i."""
    actual_w = (secrets[i] * rs[i]) % prime
    actual_u = (vs[i] * rs[i]) % prime
    return ("Verification of secret has failed:\n"
            "\t%d = %d * %d   &&   %d = %d * %d\n"
            "\t%d = %d   &&   %d = %d" % (ws[i], secrets[i], rs[i], us[i], vs[i], rs[i],
                                          ws[i], actual_w, us[i], actual_u))


class OutputDeliveryObject:
    """amphora-common/.../OutputDeliveryObject.java:55-106 (equal-length check :80-88)."""

    FIELDS = ("secret_shares", "r_shares", "v_shares", "w_shares", "u_shares")

    def __init__(self, secret_shares: bytes, r_shares: bytes, v_shares: bytes,
                 w_shares: bytes, u_shares: bytes):
        n = len(secret_shares)
        if not (len(r_shares) == n and len(v_shares) == n and len(w_shares) == n
                and len(u_shares) == n):
            raise IllegalArgumentException("The provided shares must be of the same length")
        self.secret_shares = bytes(secret_shares)
        self.r_shares = bytes(r_shares)
        self.v_shares = bytes(v_shares)
        self.w_shares = bytes(w_shares)
        self.u_shares = bytes(u_shares)

    def __eq__(self, other):
        return isinstance(other, OutputDeliveryObject) and all(
            getattr(self, f) == getattr(other, f) for f in self.FIELDS)


def verify_output_delivery_objects(util: ClientSecretShareUtil,
                                   odos: Sequence[OutputDeliveryObject]) -> List[int]:
    """DefaultAmphoraClient.verifyOutputDeliveryObjects :476-505:
    5x recombineObject then verifySecrets(secrets, rs, us, vs, ws)."""
    secrets = util.recombine_object([o.secret_shares for o in odos])
    rs = util.recombine_object([o.r_shares for o in odos])
    us = util.recombine_object([o.u_shares for o in odos])
    vs = util.recombine_object([o.v_shares for o in odos])
    ws = util.recombine_object([o.w_shares for o in odos])
    util.verify_secrets(secrets, rs, us, vs, ws)
    return secrets


def create_secret_masked_inputs(util: ClientSecretShareUtil, secrets: Sequence[int],
                                mask_odos: Sequence[OutputDeliveryObject]) -> List[bytes]:
    """DefaultAmphoraClient.createSecret :150-160 (arithmetic only):
    verify the Input Mask ODOs, then maskInput per word."""
    masks = verify_output_delivery_objects(util, mask_odos)
    return [util.mask_input(secrets[i], masks[i]) for i in range(len(secrets))]


# --------------------------------------------------------------------------
# Service side: amphora-service/.../calculation/SecretShareUtil.java
# --------------------------------------------------------------------------
def convert_to_secret_share(spdz: MpSpdzIntegrationUtils, masked_inputs: Sequence[bytes],
                            mac_key: str, input_masks: Sequence[Tuple[bytes, bytes]],
                            use_zero_input_as_data: bool) -> bytes:
    """SecretShareUtil.convertToSecretShare :58-81 + computeSecretShare :83-107.

    input_masks: per word the (value, mac) byte pair of share 0 of the tuple.
    Returns SecretShare.data (32 B per word: value || mac)."""
    if len(masked_inputs) != len(input_masks):
        raise IllegalArgumentException("Received more input data than available inputMasks.")
    zero_input = spdz.from_gfp(bytes(WORD_WIDTH))  # :44
    out = bytearray()
    for mi, (mval, mmac) in zip(masked_inputs, input_masks):
        key = int(mac_key)  # new BigInteger(mac) :86
        public_value = spdz.from_gfp(mi)
        individual = zero_input if use_zero_input_as_data else spdz.from_gfp(mi)
        share_value = spdz.from_gfp(mval)
        share_mac = spdz.from_gfp(mmac)
        out += spdz.to_gfp((share_value + individual) % spdz.prime)
        out += spdz.to_gfp((share_mac + key * public_value) % spdz.prime)
    return bytes(out)


# --------------------------------------------------------------------------
# Service side: OutputDeliveryService.java (local arithmetic only)
# --------------------------------------------------------------------------
def strip_macs(share_data: bytes) -> bytes:
    """computeOutputDeliveryObject(SecretShare, UUID) :75-86: first 16 of
    every 32 bytes."""
    n = len(share_data) // SHARE_WIDTH
    return b"".join(share_data[i * SHARE_WIDTH:i * SHARE_WIDTH + WORD_WIDTH] for i in range(n))


def parse_input_masks(stream: bytes) -> List[Tuple[bytes, bytes]]:
    """castor TupleList<InputMask> byte layout: value(16) || mac(16) per tuple."""
    return [(stream[i:i + 16], stream[i + 16:i + 32]) for i in range(0, len(stream), 32)]


def parse_triples(stream: bytes) -> List[Tuple[bytes, bytes, bytes]]:
    """castor TupleList<MultiplicationTriple>: (a, b, c) share values; MACs skipped."""
    return [(stream[i:i + 16], stream[i + 32:i + 48], stream[i + 64:i + 80])
            for i in range(0, len(stream), 96)]


def odo_factor_pairs(spdz, share_data16: bytes, masks: Sequence[Tuple[bytes, bytes]]):
    """computeOutputDeliveryObject(byte[], UUID) :121-139: raw copies of y, r, v
    and the factor pairs (y_i, r_i), (v_i, r_i) as canonical BigIntegers."""
    ws = words(share_data16)
    y_raw, r_raw, v_raw, pairs = bytearray(), bytearray(), bytearray(), []
    for i, y in enumerate(ws):
        m1 = masks[2 * i][0]
        m2 = masks[2 * i + 1][0]
        y_raw += y
        r_raw += m1
        v_raw += m2
        yb, m1b, m2b = spdz.from_gfp(y), spdz.from_gfp(m1), spdz.from_gfp(m2)
        pairs.append((yb, m1b))
        pairs.append((m2b, m1b))
    return bytes(y_raw), bytes(r_raw), bytes(v_raw), pairs


def beaver_diffs(spdz, pairs, triples) -> List[Tuple[int, int]]:
    """multiplyShares :186-200: d = x - fromGfp(a), e = y - fromGfp(b); signed,
    NOT reduced."""
    return [(x - spdz.from_gfp(t[0]), y - spdz.from_gfp(t[1])) for (x, y), t in zip(pairs, triples)]


def recombine_diffs(prime: int, diff_lists: Sequence[Sequence[Tuple[int, int]]]):
    """recombineDiffs :231-272: Future.reduce over the parties' lists with a
    pairwise ``add().mod(p)``.  A single list is returned unreduced (reduce
    of one element)."""
    acc = list(diff_lists[0])
    for nxt in diff_lists[1:]:
        acc = [((a[0] + b[0]) % prime, (a[1] + b[1]) % prime) for a, b in zip(acc, nxt)]
    return acc


def multiply_shared_secrets(spdz, triple, d: int, e: int, player_id: int) -> int:
    """multiplySharedSecrets :274-286; triple share order a=0, b=1, c=2."""
    p = spdz.prime
    share = (spdz.from_gfp(triple[2]) + d * spdz.from_gfp(triple[1])
             + e * spdz.from_gfp(triple[0])) % p
    if player_id == 0:
        share = (share + d * e) % p
    return share


def name_uuid_from_bytes(name: bytes) -> uuid.UUID:
    """java.util.UUID.nameUUIDFromBytes: MD5, version 3, IETF variant."""
    h = bytearray(hashlib.md5(name).digest())
    h[6] = (h[6] & 0x0F) | 0x30
    h[8] = (h[8] & 0x3F) | 0x80
    return uuid.UUID(bytes=bytes(h))


def operation_id(request_id: uuid.UUID, n_pairs: int) -> uuid.UUID:
    """OutputDeliveryService.java:140-141."""
    return name_uuid_from_bytes(("%s_%d" % (request_id, n_pairs)).encode())


def odo_request_id(request_id: uuid.UUID) -> uuid.UUID:
    """InputMaskCachingService.java:92-93."""
    return name_uuid_from_bytes(("%s_odo-computation" % request_id).encode())


def compute_output_delivery_object(spdz, share_data16: bytes, input_mask_stream: bytes,
                                   triple_stream: bytes, partner_diffs, player_id: int):
    """computeOutputDeliveryObject(byte[], UUID) :100-161 end to end with the
    network exchange replaced by ``partner_diffs`` (a list of the other
    parties' diff lists, in player order after this party's own).
    Returns (ODO, own diffs, products)."""
    masks = parse_input_masks(input_mask_stream)
    triples = parse_triples(triple_stream)
    y_raw, r_raw, v_raw, pairs = odo_factor_pairs(spdz, share_data16, masks)
    own = beaver_diffs(spdz, pairs, triples[:len(pairs)])
    opened = recombine_diffs(spdz.prime, [own] + list(partner_diffs))
    products = [multiply_shared_secrets(spdz, triples[k], opened[k][0], opened[k][1], player_id)
                for k in range(len(pairs))]
    w = b"".join(spdz.to_gfp(products[2 * i]) for i in range(len(pairs) // 2))
    u = b"".join(spdz.to_gfp(products[2 * i + 1]) for i in range(len(pairs) // 2))
    return OutputDeliveryObject(y_raw, r_raw, v_raw, w, u), own, products
