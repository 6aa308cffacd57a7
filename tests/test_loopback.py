"""BASELINE config C1 end to end: DefaultAmphoraClient.createSecret /
getSecret against N in-process amphora-service parties (amphora_amd.loopback)
with a fake Castor dealer -- every word of arithmetic (mask ODOs with Beaver
multiplications, client verify + masking, share conversion with MACs, share
ODOs, client recombine + verify) on the HIP kernels."""
import random
import uuid

import pytest

pytestmark = pytest.mark.gpu

from oracle import amphora_oracle as O  # noqa: E402
from tests.loopback_dealer import FakeCastor  # noqa: E402

P, R, RINV = O.TEST_PRIME, O.TEST_R, O.TEST_RINV
SPDZ = O.MpSpdzIntegrationUtils(P, R, RINV)


def _cluster(n, seed, exchange_format="json", transport="objects"):
    import torch
    assert torch.cuda.is_available()
    from amphora_amd.loopback import AmphoraParty, ExchangeHub, LoopbackAmphoraClient
    rng = random.Random(seed)
    keys = [rng.randrange(P) for _ in range(n)]
    castor = FakeCastor(P, R, RINV, keys, seed)
    hub = ExchangeHub(n)
    parties = [AmphoraParty(j, P, R, RINV, keys[j], castor, hub, exchange_format=exchange_format)
               for j in range(n)]
    return LoopbackAmphoraClient(parties, P, R, RINV, transport=transport), parties, keys, castor


@pytest.mark.parametrize("n,W,fmt,transport", [(2, 1000, "json", "objects"), (3, 257, "json", "objects"),
                                               (2, 1, "json", "objects"), (2, 1000, "objects", "objects"),
                                               (3, 257, "objects", "objects"), (2, 1000, "json", "json"),
                                               (3, 769, "json", "json"), (2, 1, "json", "json"),
                                               (4, 2, "objects", "json"), (2, 1000, "session", "objects"),
                                               (3, 769, "session", "json"), (2, 1, "session", "json"),
                                               (5, 129, "session", "json"), (16, 33, "json", "json")])
def test_upload_download_roundtrip(n, W, fmt, transport):
    """fmt: the inter-VCP open carries MultiplicationExchangeObject JSON bodies
    (GPU-coded) or in-memory FactorPair lists.  transport="json": the
    client-party hops carry the REST JSON bodies and the client runs the fused
    wire kernels (K_RV / K_MASK straight from the base64 text)."""
    import amphora_amd as A
    client, parties, keys, castor = _cluster(n, seed=W + n, exchange_format=fmt, transport=transport)
    rng = random.Random(5)
    data = [rng.randrange(2 ** 63) if i % 2 else rng.randrange(P) for i in range(W)]
    sid = client.create_secret(A.Secret.of([("k", "v")], data))
    got = client.get_secret(sid)
    assert got.data == data
    # stored shares carry valid SPDZ MACs: sum(mac) == alpha * sum(value)
    alpha = sum(keys) % P
    for i in range(W):
        val = sum(SPDZ.from_gfp(p.secrets[sid].data[32 * i:32 * i + 16]) for p in parties) % P
        mac = sum(SPDZ.from_gfp(p.secrets[sid].data[32 * i + 16:32 * i + 32]) for p in parties) % P
        assert val == data[i] % P and mac == alpha * val % P
    # tuple requests follow the reference's ids (InputMaskCachingService :92-93,
    # OutputDeliveryService :140-141)
    odo_req = O.odo_request_id(sid)
    assert any(c[1] == odo_req for c in castor.calls)
    assert any(c[1] == O.operation_id(odo_req, 2 * W) for c in castor.calls)
    if fmt in ("json", "session"):  # the last open each party sent is a well-formed body
        import json
        body = json.loads(parties[0].odo_service.last_exchange_object)
        assert list(body) == ["operationId", "playerId", "interimValues"]
        assert len(body["interimValues"]) == 2 * W and body["playerId"] == 0
    client.close()


def test_session_and_per_call_parties_interoperate():
    """A party running its requests as device-resident sessions and one running
    the per-call path send each other the same JSON bodies."""
    import amphora_amd as A
    from amphora_amd.loopback import AmphoraParty, ExchangeHub, LoopbackAmphoraClient
    rng = random.Random(77)
    keys = [rng.randrange(P) for _ in range(3)]
    castor = FakeCastor(P, R, RINV, keys, 77)
    hub = ExchangeHub(3)
    parties = [AmphoraParty(j, P, R, RINV, keys[j], castor, hub, exchange_format=fmt)
               for j, fmt in enumerate(["session", "json", "session"])]
    client = LoopbackAmphoraClient(parties, P, R, RINV, transport="json")
    data = [rng.randrange(P) for _ in range(333)]
    sid = client.create_secret(A.Secret.of([], data))
    assert client.get_secret(sid).data == data
    assert parties[0].odo_service.last_exchange_object.startswith(b'{"operationId":')
    client.close()


@pytest.mark.parametrize("transport", ["objects", "json"])
def test_tampered_party_is_detected(transport):
    import amphora_amd as A
    client, parties, _, _ = _cluster(2, seed=9, transport=transport)
    data = list(range(1, 101))
    sid = client.create_secret(A.Secret.of([], data))
    victim = parties[1]
    orig = victim.get_secret_share

    def tampered(secret_id, request_id):
        odo = orig(secret_id, request_id)
        y = bytearray(odo.secret_shares)
        y[16 * 42] ^= 0x01  # a malicious party shifts one secret share
        return A.OutputDeliveryObject(bytes(y), odo.r_shares, odo.v_shares, odo.w_shares, odo.u_shares)

    victim.get_secret_share = tampered
    with pytest.raises(A.IntegrityVerificationException, match="^Verification of secret has failed"):
        client.get_secret(sid)
    client.close()


def test_upload_without_masks_fails():
    import amphora_amd as A
    client, parties, _, _ = _cluster(2, seed=3)
    mi = A.MaskedInput(uuid.uuid4(), [A.MaskedInputData.of(bytes(16))], [])
    with pytest.raises(A.AmphoraServiceException, match="No input masks found"):
        parties[0].upload_masked_input(mi)
    client.close()


def test_party_failures_map_to_client_exceptions():
    """DefaultAmphoraClientTest.java:237-252,273-288: a failing party surfaces
    as AmphoraClientException with the reference's message shapes."""
    import amphora_amd as A
    client, parties, _, _ = _cluster(2, seed=11)
    sid = client.create_secret(A.Secret.of([], [42, 24]))
    orig = parties[1].get_secret_share

    def failing(*a):
        raise Exception("Call failed")

    parties[1].get_secret_share = failing
    with pytest.raises(A.AmphoraClientException) as ei:
        client.get_secret(sid)
    assert str(ei.value).startswith("Error(s) occurred while processing responses")
    assert "Call failed" in str(ei.value)
    parties[1].get_secret_share = orig
    assert client.get_secret(sid).data == [42, 24]
    up = parties[1].upload_masked_input
    parties[1].upload_masked_input = lambda mi: (_ for _ in ()).throw(Exception(500))
    with pytest.raises(A.AmphoraClientException) as ei:
        client.create_secret(A.Secret.of([], [7]))
    assert str(ei.value).endswith('Request for endpoint "loopback://amphora-1" failed: 500')
    parties[1].upload_masked_input = up
    client.close()


def test_partner_never_answers():
    """OutputDeliveryServiceTest.java:211-283: the open times out ->
    AmphoraServiceException("Failed to open values for operation #...")."""
    import amphora_amd as A
    from amphora_amd.loopback import AmphoraParty, ExchangeHub
    rng = random.Random(4)
    keys = [rng.randrange(P) for _ in range(2)]
    castor = FakeCastor(P, R, RINV, keys, 4)
    hub = ExchangeHub(2, timeout_s=0.5)
    p0 = AmphoraParty(0, P, R, RINV, keys[0], castor, hub)
    with pytest.raises(A.AmphoraServiceException, match="^Failed to open values for operation #"):
        p0.get_input_masks(uuid.uuid4(), 10)
