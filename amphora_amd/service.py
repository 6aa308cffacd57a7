"""Host-side mirror of the party (amphora-service) arithmetic, routed to the
HIP kernels through the C ABI.

Mirrors:
* calculation/SecretShareUtil.convertToSecretShare
      amphora-service/.../calculation/SecretShareUtil.java:30-107     (K_CONV)
* calculation/OutputDeliveryService.computeOutputDeliveryObject
      amphora-service/.../calculation/OutputDeliveryService.java:57-286
      local parts: K_ODO_PRE -> exchange -> open (recombineDiffs) + K_ODO_POST,
      the last two fused in one launch (amph_open_post)
* persistence/cache/InputMaskCachingService.getInputMasksAsOutputDeliveryObject
      InputMaskCachingService.java:77-99 (value halves of the mask tuples)

Castor, Redis and the inter-VCP HTTP exchange are out of scope:
they are injected as callables, exactly where the reference's tests mock them
(OutputDeliveryServiceTest.java:183-209).
"""
from __future__ import annotations

import hashlib
import uuid
from typing import Callable, List, Sequence

import numpy as np

from . import _lib
from .client import pack, unpack
from .entities import (AmphoraServiceException, FactorPair, IllegalArgumentException,
                       MaskedInput, MultiplicationExchangeObject, OutputDeliveryObject,
                       SecretShare, SHARE_WIDTH, WORD_WIDTH)

INPUT_MASK_GFP = "INPUT_MASK_GFP"  # castor TupleType; tuple = value(16) || mac(16)
MULTIPLICATION_TRIPLE_GFP = "MULTIPLICATION_TRIPLE_GFP"  # a,mac,b,mac,c,mac (96 B)
TUPLE_SIZE = {INPUT_MASK_GFP: 32, MULTIPLICATION_TRIPLE_GFP: 96}


def name_uuid_from_bytes(name: bytes) -> uuid.UUID:
    """java.util.UUID.nameUUIDFromBytes (MD5, version 3)."""
    h = bytearray(hashlib.md5(name).digest())
    h[6] = (h[6] & 0x0F) | 0x30
    h[8] = (h[8] & 0x3F) | 0x80
    return uuid.UUID(bytes=bytes(h))


class SecretShareUtil:
    """Service-side SecretShareUtil (constructed from the SPDZ context)."""

    def __init__(self, ctx: _lib.Context):
        self._ctx = ctx

    def convert_to_secret_share(self, masked_input: MaskedInput, mac_key: str, input_masks,
                                use_zero_input_as_data: bool) -> SecretShare:
        """convertToSecretShare :58-81.  input_masks: the tuple stream
        (W x 32 B: share-0 value || mac) or a list of (value, mac) pairs."""
        masks = _tuples(input_masks, 32)
        if len(masked_input.data) != masks.shape[0]:
            raise IllegalArgumentException("Received more input data than available inputMasks.")
        data = masked_input.data
        if hasattr(data, "words"):  # MaskedInputWords: the array itself
            masked = data.words
        else:
            masked = np.frombuffer(b"".join(d.value for d in data), np.uint8).reshape(-1, 16) \
                if data else np.zeros((0, 16), np.uint8)
        key = int(mac_key) % self._ctx.prime  # new BigInteger(mac) :86 (used mod p)
        out = self._ctx.convert_share(masked, masks, key, use_zero_input_as_data)
        return SecretShare(masked_input.secret_id, out.tobytes(), list(masked_input.tags))


def _tuples(x, size):
    if isinstance(x, (list, tuple)):
        x = b"".join(bytes(a) + bytes(b) for a, b in x) if x and isinstance(x[0], tuple) else b"".join(x)
    return _lib.words_view(x, size)


def encode_diffs(pairs: Sequence[FactorPair]):
    """FactorPair list (signed BigIntegers, |x| < 2^128) -> (mag, neg) arrays."""
    mags, negs = bytearray(), bytearray()
    for fp in pairs:
        for x in (fp.a, fp.b):
            mags += abs(int(x)).to_bytes(16, "little")
            negs.append(1 if x < 0 else 0)
    n = len(pairs)
    return (np.frombuffer(bytes(mags), np.uint8).reshape(n, 2, 16).copy(),
            np.frombuffer(bytes(negs), np.uint8).reshape(n, 2).copy())


def decode_diffs(mag, neg) -> List[FactorPair]:
    vals = unpack(np.ascontiguousarray(mag).reshape(-1, 16))
    sg = np.ascontiguousarray(neg).reshape(-1).tolist()
    signed = [-v if s else v for v, s in zip(vals, sg)]
    return [FactorPair(signed[2 * k], signed[2 * k + 1]) for k in range(len(signed) // 2)]


def _check_partner(m, own):
    """A partner must open exactly as many FactorPairs as this party did: the
    reference's recombineDiffs reads every partner's list at each own index
    (:231-272) and fails inside the open's Try on a short one."""
    if tuple(m.shape) != tuple(own.shape):
        raise ValueError("partner opened %d pairs, expected %d" % (m.shape[0], own.shape[0]))


class OutputDeliveryService:
    """OutputDeliveryService with Castor and the inter-VCP open injected.

    tuple_source(request_id, tuple_type, count) -> bytes   (Castor download)
    exchange(MultiplicationExchangeObject) -> list of the partners' FactorPair
        lists in player order (open + Redis gather, recombineDiffs :231-272)

    exchange_format="json": the exchange carries the MultiplicationExchangeObject
    as its /inter-vcp/open JSON body (bytes in, partners' bodies out), coded on
    the GPU (amph_exchange_*) -- no per-value Python objects.
    exchange_format="session": the same JSON bodies, with the request run as a
    device-resident party session (amph_party_*): the triples and every party's
    diffs stay on the GPU between the open's two halves (needs n_parties).
    """

    def __init__(self, ctx: _lib.Context, player_id: int,
                 tuple_source: Callable[[uuid.UUID, str, int], bytes],
                 exchange: Callable, exchange_format: str = "objects", n_parties: int = None):
        if exchange_format not in ("objects", "json", "session"):
            raise ValueError("exchange_format must be 'objects', 'json' or 'session'")
        if exchange_format == "session" and not n_parties:
            raise ValueError("exchange_format='session' needs n_parties")
        self._ctx = ctx
        self.player_id = player_id
        self._tuples = tuple_source
        self._exchange = exchange
        self._json = exchange_format == "json"
        self._session = exchange_format == "session"
        self.n_parties = n_parties
        self.last_exchange_object = None

    def _download(self, request_id, tuple_type, count):
        try:
            data = self._tuples(request_id, tuple_type, count)
        except Exception as e:  # Try.of(..).getOrElseThrow :103-107, :178-185
            raise AmphoraServiceException("Failed to retrieve the required Tuples form Castor") from e
        try:
            tuples = _lib.words_view(data, TUPLE_SIZE[tuple_type])
        except ValueError as e:
            raise AmphoraServiceException("Castor returned a malformed %s stream" % tuple_type) from e
        if tuples.shape[0] != count:
            # the reference indexes tripleShares.get(i) / inputMasks.get(2i+1) and
            # fails with IndexOutOfBounds on a short list (:121-139, :186-200); the
            # kernels take one word count and cannot see a short buffer, so the
            # stream's length is checked before any launch
            raise AmphoraServiceException("Castor returned %d %s tuples, %d requested"
                                          % (tuples.shape[0], tuple_type, count))
        return tuples

    def compute_output_delivery_object(self, share, request_id: uuid.UUID) -> OutputDeliveryObject:
        """computeOutputDeliveryObject(SecretShare | byte[], UUID) :75-161."""
        if isinstance(share, SecretShare):
            data, stride = share.data, SHARE_WIDTH  # MACs stripped inside K_ODO_PRE (:79-84)
        else:
            data, stride = bytes(share), WORD_WIDTH
        return self._compute(_lib.words_view(data, stride), stride, request_id)

    def _compute(self, share_words, stride, request_id):
        W = share_words.shape[0]
        masks = self._download(request_id, INPUT_MASK_GFP, 2 * W)
        op_id = name_uuid_from_bytes(("%s_%d" % (request_id, 2 * W)).encode())  # :140-141
        triples = self._download(op_id, MULTIPLICATION_TRIPLE_GFP, 2 * W)
        if self._session:
            return self._compute_session(share_words, stride, masks, triples, op_id)
        y, r, v, mag, neg = self._ctx.odo_pre(share_words, stride, masks, triples)
        mags, negs = [mag], [neg]
        if self._json:
            from . import wire
            own = wire.exchange_to_json(self._ctx, op_id, self.player_id, mag, neg)
            self.last_exchange_object = own
            try:
                partners = self._exchange(own)
                for body in partners:
                    p_op, _, m, n = wire.exchange_from_json(self._ctx, body, mag.shape[0])
                    if p_op != op_id:
                        raise ValueError("operation id %s != %s" % (p_op, op_id))
                    _check_partner(m, mag)
                    mags.append(m)
                    negs.append(n)
            except Exception as e:
                raise AmphoraServiceException("Failed to open values for operation #%s" % op_id) from e
        else:
            xo = MultiplicationExchangeObject(op_id, self.player_id, decode_diffs(mag, neg))
            self.last_exchange_object = xo
            try:
                partners = self._exchange(xo)
                for lst in partners:  # recombineDiffs runs inside the same Try (:205-219)
                    m, n = encode_diffs(lst)
                    _check_partner(m, mag)
                    mags.append(m)
                    negs.append(n)
            except Exception as e:
                raise AmphoraServiceException("Failed to open values for operation #%s" % op_id) from e
        # recombineDiffs (:231-272) + multiplySharedSecrets (:274-286) + the w/u
        # encoding (:147-152), one launch: the opened values stay on chip
        w, u = self._ctx.open_post(mags, negs, triples, self.player_id == 0)
        return OutputDeliveryObject(y.tobytes(), r.tobytes(), v.tobytes(), w.tobytes(), u.tobytes())

    def _compute_session(self, share_words, stride, masks, triples, op_id):
        """_compute with the tuples, diffs and ODO fields device-resident
        (amph_party_begin -> the own body -> each partner's interimValues ->
        amph_party_finish); same results, bit for bit."""
        from . import wire
        with self._ctx.party_begin(share_words, stride, masks, triples, self.n_parties) as s:
            own = wire.exchange_body(op_id, self.player_id, s.text())
            self.last_exchange_object = own
            try:
                partners = self._exchange(own)
                if len(partners) != self.n_parties - 1:
                    raise ValueError("%d partner bodies, %d expected" % (len(partners), self.n_parties - 1))
                for slot, body in enumerate(partners, start=1):
                    body = bytes(body)
                    p_op, _, lb, rb = wire.exchange_span(body)
                    if p_op != op_id:
                        raise ValueError("operation id %s != %s" % (p_op, op_id))
                    s.partner(slot, body[lb:rb + 1])
            except Exception as e:
                raise AmphoraServiceException("Failed to open values for operation #%s" % op_id) from e
            w, u = s.finish(self.player_id == 0)
            return OutputDeliveryObject(s.y.tobytes(), s.r.tobytes(), s.v.tobytes(), w.tobytes(), u.tobytes())

    def get_input_masks_as_output_delivery_object(self, request_id: uuid.UUID, count: int):
        """InputMaskCachingService.getInputMasksAsOutputDeliveryObject :77-99:
        the mask tuples' value halves (stride 32) feed the ODO computation
        under odoRequestId = nameUUIDFromBytes(requestId + "_odo-computation").
        Returns (ODO, the mask tuple stream to cache)."""
        masks = self._download(request_id, INPUT_MASK_GFP, count)
        odo_req = name_uuid_from_bytes(("%s_odo-computation" % request_id).encode())
        return self._compute(masks, 32, odo_req), masks
