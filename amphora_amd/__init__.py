"""amphora_amd -- MI355X-native share arithmetic for Carbyne Stack Amphora.

The hot path (Input Supply masking, Output Delivery recombine + MAC verify,
and the party-side share conversion / ODO arithmetic) runs as hand-written
gfx950 HIP kernels in libamphora_hip.so behind the C ABI of
include/amphora.h.  This package is the host-side mirror of the reference's
Java interface (client.SecretShareUtil, service.SecretShareUtil,
service.OutputDeliveryService) on top of that ABI.  Importing it loads the
native library and raises if it is missing: there is no CPU fallback.
"""
from . import _lib  # noqa: F401  (loads libamphora_hip.so or raises)
from ._lib import Context, AmphoraNativeError  # noqa: F401
from .entities import (AmphoraClientException, AmphoraServiceException, FactorPair, IllegalArgumentException,  # noqa: F401
                       IntegrityVerificationException, MaskedInput, MaskedInputData,
                       MultiplicationExchangeObject, OutputDeliveryObject, Secret, SecretShare)

__version__ = "0.1.0"
