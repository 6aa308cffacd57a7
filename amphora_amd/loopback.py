"""In-process N-party loopback of Amphora's upload / download protocol.

Replaces the HTTP hops of the reference with direct calls while keeping the
call sequence of its controllers and services, so BASELINE config C1
("1k-word secret upload+download via DefaultAmphoraClient against 2 loopback
amphora-service parties") runs end to end on the HIP kernels:

upload  DefaultAmphoraClient.createSecret            DefaultAmphoraClient.java:150-170
          -> GET /input-masks                          InputMaskShareController.java:35-43
             InputMaskCachingService.getInputMasksAsOutputDeliveryObject  :77-99
             (OutputDeliveryService: K_ODO_PRE -> open -> K_ODO_POST)
          -> client verify + mask (K_MASK)
          -> POST /masked-inputs                       MaskedInputController.java:53-68
             StorageService.createSecret :95-117 -> convertToSecretShare (K_CONV)
download DefaultAmphoraClient.getSecret               DefaultAmphoraClient.java:206-217
          -> GET /secret-shares/{id}?requestId         SecretShareController.java:110-124
             OutputDeliveryService.computeOutputDeliveryObject(SecretShare)
          -> client recombine + verify (K_RV)

The inter-VCP open (DefaultAmphoraInterVcpClient.open + the Redis mailbox of
InterimValueCachingService, OutputDeliveryService.java:201-272) is the
ExchangeHub below; parties run concurrently in threads, as the services do.
The tuple source (Castor) is injected: any callable
``(player_id, request_id, tuple_type, count) -> bytes``.
"""
from __future__ import annotations

import threading
import uuid
from concurrent.futures import ThreadPoolExecutor
from typing import Callable, Dict, List, Sequence

from . import _lib
from .client import (SecretShareUtil, create_masked_input, create_masked_input_json,
                     verify_output_delivery_objects, verify_vss_json)
from .entities import (AmphoraClientException, AmphoraServiceException, FactorPair, MaskedInput,
                       MultiplicationExchangeObject, OutputDeliveryObject, Secret, SecretShare)
from .service import INPUT_MASK_GFP, OutputDeliveryService
from .service import SecretShareUtil as ServiceSecretShareUtil

NO_INPUT_MASKS_FOUND_FOR_REQUEST_ID_EXCEPTION_MSG = "No input masks found for request ID %s"
REQUEST_FOR_ENDPOINT_FAILED_EXCEPTION_MSG = 'Request for endpoint "%s" failed: %s'  # DefaultAmphoraClient.java:81-82


class ExchangeHub:
    """Mailbox for MultiplicationExchangeObjects keyed by (operationId,
    playerId) -- the Redis store + inter-VCP open of the reference.  Each
    party posts its own diffs and waits (bounded) for every other party's."""

    def __init__(self, n_parties: int, timeout_s: float = 30.0):
        self.n = n_parties
        self.timeout_s = timeout_s
        self._box: Dict[uuid.UUID, Dict[int, List[FactorPair]]] = {}
        self._cv = threading.Condition()

    def exchange(self, xo):
        """xo: a MultiplicationExchangeObject (-> partners' FactorPair lists)
        or its JSON body (-> partners' JSON bodies, as POSTed to /inter-vcp/open)."""
        if isinstance(xo, MultiplicationExchangeObject):
            op, pid, item = xo.operation_id, xo.player_id, list(xo.interim_values)
        else:
            from .wire import exchange_header
            item = bytes(xo)
            op, pid = exchange_header(item)
        with self._cv:
            self._box.setdefault(op, {})[pid] = item
            self._cv.notify_all()
            ok = self._cv.wait_for(lambda: len(self._box[op]) == self.n, timeout=self.timeout_s)
            if not ok:
                raise TimeoutError("partner diffs for operation %s not received" % op)
            box = self._box[op]
            return [box[p] for p in sorted(box) if p != pid]


class AmphoraParty:
    """One amphora-service (VCP) with its MAC key share, tuple source, input
    mask cache (Redis) and secret store (Postgres/MinIO), all in memory."""

    def __init__(self, player_id: int, prime: int, r: int, r_inv: int, mac_key: int,
                 tuple_source: Callable[[int, uuid.UUID, str, int], bytes], hub: ExchangeHub,
                 device: int = 0, exchange_format: str = "json"):
        self.player_id = player_id
        self.ctx = _lib.Context(prime, r, r_inv, device)
        self.mac_key = mac_key
        self._castor = lambda rid, ttype, count: tuple_source(player_id, rid, ttype, count)
        self.odo_service = OutputDeliveryService(self.ctx, player_id, self._castor, hub.exchange,
                                                 exchange_format, n_parties=hub.n)
        self.share_util = ServiceSecretShareUtil(self.ctx)
        self.input_mask_store: Dict[uuid.UUID, object] = {}
        self.secrets: Dict[uuid.UUID, SecretShare] = {}

    # GET /input-masks?requestId&count
    def get_input_masks(self, request_id: uuid.UUID, count: int) -> OutputDeliveryObject:
        odo, masks = self.odo_service.get_input_masks_as_output_delivery_object(request_id, count)
        self.input_mask_store[request_id] = masks  # ops.set(cachePrefix + requestId, ...)
        return odo

    # POST /masked-inputs
    def upload_masked_input(self, masked_input: MaskedInput) -> uuid.UUID:
        masks = self.input_mask_store.get(masked_input.secret_id)
        if masks is None:
            raise AmphoraServiceException(
                NO_INPUT_MASKS_FOUND_FOR_REQUEST_ID_EXCEPTION_MSG % masked_input.secret_id)
        share = self.share_util.convert_to_secret_share(
            masked_input, str(self.mac_key), masks, self.player_id != 0)
        self.secrets[masked_input.secret_id] = share
        del self.input_mask_store[masked_input.secret_id]
        return masked_input.secret_id

    # GET /secret-shares/{id}?requestId
    def get_secret_share(self, secret_id: uuid.UUID, request_id: uuid.UUID) -> OutputDeliveryObject:
        return self.odo_service.compute_output_delivery_object(self.secrets[secret_id], request_id)


class LoopbackAmphoraClient:
    """DefaultAmphoraClient over in-process parties (transport = direct calls,
    fanned out concurrently like AmphoraCommunicationClient's parallelStream)."""

    def __init__(self, parties: Sequence[AmphoraParty], prime: int, r: int, r_inv: int,
                 device: int = 0, transport: str = "objects"):
        """transport="json": every hop carries the JSON body the REST API
        would (OutputDeliveryObject / VerifiableSecretShare / MaskedInput,
        base64 coded on the parties' GPUs), and the client consumes and
        produces the text with the fused wire kernels (client.verify_vss_json,
        client.create_masked_input_json)."""
        if transport not in ("objects", "json"):
            raise ValueError("transport must be 'objects' or 'json'")
        self.parties = list(parties)
        self.util = SecretShareUtil.of(prime, r, r_inv, device)
        self.transport = transport
        self._pool = ThreadPoolExecutor(max_workers=len(self.parties))

    @staticmethod
    def uri(party) -> str:
        return "loopback://amphora-%d" % party.player_id

    def _fan_out(self, fn):
        """One Try per party, like AmphoraCommunicationClient's results map."""
        futs = [self._pool.submit(fn, p) for p in self.parties]
        out = []
        for p, f in zip(self.parties, futs):
            try:
                out.append((p, f.result(), None))
            except Exception as e:  # noqa: BLE001 -- a failed request, reported below
                out.append((p, None, e))
        return out

    @staticmethod
    def _unwrap(tries):
        """DefaultAmphoraClient.unwrap :693-711."""
        failures = [e for _, _, e in tries if e is not None]
        if failures:
            raise AmphoraClientException("Error(s) occurred while processing responses:\n\t%s"
                                         % "\n\t".join(str(e) for e in failures))
        return [v for _, v, _ in tries]

    def _check_success(self, tries):
        """DefaultAmphoraClient.checkSuccess :613-638."""
        failed = [(p, e) for p, _, e in tries if e is not None]
        if failed:
            msg = "Secret could not be created due to http errors returned by the following providers: "
            for p, e in failed:
                msg += "\n\t" + REQUEST_FOR_ENDPOINT_FAILED_EXCEPTION_MSG % (self.uri(p), e)
            raise AmphoraClientException(msg)

    def create_secret(self, secret: Secret) -> uuid.UUID:
        if self.transport == "json":
            from . import wire
            bodies = self._unwrap(self._fan_out(lambda p: wire.odo_to_json(
                p.ctx, p.get_input_masks(secret.secret_id, secret.size()))))
            text = create_masked_input_json(self.util, secret, bodies)
            self._check_success(self._fan_out(
                lambda p: p.upload_masked_input(wire.masked_input_from_json(p.ctx, text))))
            return secret.secret_id
        odos = self._unwrap(self._fan_out(lambda p: p.get_input_masks(secret.secret_id, secret.size())))
        masked = create_masked_input(self.util, secret, odos)
        self._check_success(self._fan_out(lambda p: p.upload_masked_input(masked)))
        return secret.secret_id

    def get_secret(self, secret_id: uuid.UUID) -> Secret:
        request_id = uuid.uuid4()
        if self.transport == "json":
            from . import wire
            bodies = self._unwrap(self._fan_out(lambda p: wire.vss_to_json(
                p.ctx, secret_id, p.secrets[secret_id].tags, p.get_secret_share(secret_id, request_id),
                pretty=False)))
            sid, tags, data = verify_vss_json(self.util, bodies, secret_id)
            return Secret(sid, tags, data)
        odos = self._unwrap(self._fan_out(lambda p: p.get_secret_share(secret_id, request_id)))
        data = verify_output_delivery_objects(self.util, odos)
        return Secret(secret_id, list(self.parties[0].secrets[secret_id].tags), data)

    def close(self):
        self._pool.shutdown()
