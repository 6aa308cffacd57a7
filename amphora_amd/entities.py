"""Wire entities of the hot path (amphora-common), with the reference's
length invariants and exception messages.

* OutputDeliveryObject   amphora-common/.../OutputDeliveryObject.java:55-106
* MaskedInputData        amphora-common/.../MaskedInputData.java:24-52
* MaskedInput            amphora-common/.../MaskedInput.java:25-62
* SecretShare            amphora-common/.../SecretShare.java:39-88
* FactorPair             amphora-common/.../FactorPair.java:17-25
* MultiplicationExchangeObject  amphora-common/.../MultiplicationExchangeObject.java:19-39
* Secret                 amphora-java-client/.../Secret.java:20-65
* exceptions             amphora-common/.../exceptions/*.java
"""
from __future__ import annotations

import uuid
from dataclasses import dataclass, field
from collections.abc import Sequence
from typing import List, Optional

WORD_WIDTH = 16
SHARE_WIDTH = 32


class IntegrityVerificationException(RuntimeError):
    """IntegrityVerificationException.java:15-26 (a RuntimeException)."""


class IllegalArgumentException(ValueError):
    """java.lang.IllegalArgumentException as thrown on the path."""


class NullPointerException(TypeError):
    """java.lang.NullPointerException from lombok @NonNull, same message."""


class AmphoraServiceException(RuntimeError):
    """AmphoraServiceException.java:16-37."""


class AmphoraClientException(Exception):
    """AmphoraClientException (amphora-java-client): a failed request to at
    least one party (DefaultAmphoraClient.java:613-638, 693-728)."""


class OutputDeliveryObject:
    FIELDS = ("secret_shares", "r_shares", "v_shares", "w_shares", "u_shares")

    def __init__(self, secret_shares, r_shares, v_shares, w_shares, u_shares):
        arrays = [bytes(x) if not hasattr(x, "is_cuda") else x
                  for x in (secret_shares, r_shares, v_shares, w_shares, u_shares)]
        n = [_nbytes(a) for a in arrays]
        if any(x is None for x in arrays):
            raise TypeError("shares must not be null")
        if any(k != n[0] for k in n[1:]):
            raise IllegalArgumentException("The provided shares must be of the same length")
        (self.secret_shares, self.r_shares, self.v_shares, self.w_shares,
         self.u_shares) = arrays

    def fields(self):
        return (self.secret_shares, self.r_shares, self.v_shares, self.w_shares, self.u_shares)

    def __eq__(self, other):
        return isinstance(other, OutputDeliveryObject) and all(
            bytes(a) == bytes(b) for a, b in zip(self.fields(), other.fields()))

    def __repr__(self):
        return "OutputDeliveryObject(%d words)" % (_nbytes(self.secret_shares) // WORD_WIDTH)


def _nbytes(a) -> int:
    if hasattr(a, "nbytes"):
        return int(a.nbytes) if not hasattr(a, "element_size") else a.numel() * a.element_size()
    return len(a)


@dataclass(frozen=True)
class MaskedInputData:
    value: bytes

    @staticmethod
    def of(value: bytes) -> "MaskedInputData":
        if value is None or len(value) != WORD_WIDTH:
            raise IllegalArgumentException(
                "Length of a Masked Input value has to be %d bytes." % WORD_WIDTH)
        return MaskedInputData(bytes(value))


class MaskedInputWords(Sequence):
    """List<MaskedInputData> backed by one (W, 16) uint8 array: the masked
    words as the kernels write them, materialised as MaskedInputData only
    when an element is read (the host mirror hands the array itself to the
    next kernel or codec instead of W Python objects)."""

    def __init__(self, words):
        import numpy as np
        w = np.ascontiguousarray(words, np.uint8)
        if w.ndim != 2 or w.shape[1] != WORD_WIDTH:
            raise IllegalArgumentException(
                "Length of a Masked Input value has to be %d bytes." % WORD_WIDTH)
        self.words = w

    def __len__(self):
        return self.words.shape[0]

    def __getitem__(self, i):
        if isinstance(i, slice):
            return MaskedInputWords(self.words[i])
        return MaskedInputData(self.words[i].tobytes())

    def __eq__(self, other):
        return list(self) == list(other)


@dataclass
class MaskedInput:
    """MaskedInput.java:25-62: secretId and data non-null; null tags become an
    empty list (MaskedInputTest.java)."""
    secret_id: uuid.UUID
    data: List[MaskedInputData]
    tags: list = field(default_factory=list)

    def __post_init__(self):
        for name in ("secret_id", "data"):
            if getattr(self, name) is None:
                raise NullPointerException("%s is marked non-null but is null"
                                           % ("secretId" if name == "secret_id" else name))
        if self.tags is None:
            self.tags = []


INVALID_LENGTH_EXCEPTION_MSG = "Length of a SecretShare's data must e a multiple of %s bytes!"


@dataclass
class SecretShare:
    secret_id: Optional[uuid.UUID]
    data: bytes
    tags: list = field(default_factory=list)

    def __post_init__(self):
        if len(self.data) % SHARE_WIDTH != 0:
            raise IllegalArgumentException(INVALID_LENGTH_EXCEPTION_MSG % SHARE_WIDTH)


@dataclass(frozen=True)
class FactorPair:
    a: int
    b: int

    @staticmethod
    def of(a: int, b: int) -> "FactorPair":
        return FactorPair(a, b)


@dataclass
class MultiplicationExchangeObject:
    operation_id: uuid.UUID
    player_id: int
    interim_values: List[FactorPair]


@dataclass
class Secret:
    secret_id: Optional[uuid.UUID]
    tags: list
    data: List[int]

    @staticmethod
    def of(tags, data, secret_id=None) -> "Secret":
        return Secret(secret_id or uuid.uuid4(), list(tags), list(data))

    def size(self) -> int:
        return len(self.data)
