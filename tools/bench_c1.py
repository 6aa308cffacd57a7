"""BASELINE config C1: a 1k-word secret upload + download through the
client against 2 in-process parties (amphora_amd.loopback), every word of
arithmetic on the GPU, the inter-VCP opens as MultiplicationExchangeObject
JSON.  Reports the upload and download latencies; the fake Castor dealer
(Python tuple generation, test infrastructure) generates each request's
tuples before the timed call.

    python tools/bench_c1.py [--words 1000] [--reps 20] [--transport objects|json]

--transport json: the client-party hops carry the REST JSON bodies and the
client runs K_RV / K_MASK straight from the base64 text.
"""
import argparse
import json
import os
import random
import statistics
import sys
import time
import uuid

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--words", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--parties", type=int, default=2)
    ap.add_argument("--transport", choices=["objects", "json"], default="objects")
    a = ap.parse_args()
    import amphora_amd as A
    from amphora_amd.loopback import AmphoraParty, ExchangeHub, LoopbackAmphoraClient
    from amphora_amd.spdz import TEST_PRIME, TEST_R, TEST_RINV
    from tests.loopback_dealer import FakeCastor
    P, R, RINV = TEST_PRIME, TEST_R, TEST_RINV
    rng = random.Random(1)
    keys = [rng.randrange(P) for _ in range(a.parties)]
    castor = FakeCastor(P, R, RINV, keys, 1)
    hub = ExchangeHub(a.parties)
    parties = [AmphoraParty(j, P, R, RINV, keys[j], castor, hub) for j in range(a.parties)]
    client = LoopbackAmphoraClient(parties, P, R, RINV, transport=a.transport)
    data = [rng.randrange(2 ** 63) for _ in range(a.words)]
    W = a.words
    from amphora_amd import loopback as LB
    from amphora_amd.service import INPUT_MASK_GFP, MULTIPLICATION_TRIPLE_GFP, name_uuid_from_bytes

    def prewarm(request_ids):
        # the dealer caches each (requestId, tupleType); generating here keeps
        # its Python tuple generation out of the timed calls
        for rid, ttype, count in request_ids:
            for j in range(a.parties):
                castor(j, rid, ttype, count)

    def ids_upload(sid):
        odo_req = name_uuid_from_bytes(("%s_odo-computation" % sid).encode())
        op = name_uuid_from_bytes(("%s_%d" % (odo_req, 2 * W)).encode())
        return [(sid, INPUT_MASK_GFP, W), (odo_req, INPUT_MASK_GFP, 2 * W), (op, MULTIPLICATION_TRIPLE_GFP, 2 * W)]

    def ids_download(req):
        op = name_uuid_from_bytes(("%s_%d" % (req, 2 * W)).encode())
        return [(req, INPUT_MASK_GFP, 2 * W), (op, MULTIPLICATION_TRIPLE_GFP, 2 * W)]

    up, down = [], []
    real_uuid4 = LB.uuid.uuid4
    for rep in range(a.reps + 2):
        sid, req = uuid.uuid4(), uuid.uuid4()
        prewarm(ids_upload(sid) + ids_download(req))
        LB.uuid.uuid4 = lambda: req  # get_secret's request id, known to the prewarm
        try:
            t0 = time.perf_counter()
            client.create_secret(A.Secret(sid, [("k", "v")], data))
            t1 = time.perf_counter()
            got = client.get_secret(sid)
            t2 = time.perf_counter()
        finally:
            LB.uuid.uuid4 = real_uuid4
        assert [int(x) for x in got.data] == data
        if rep >= 2:
            up.append((t1 - t0) * 1e3)
            down.append((t2 - t1) * 1e3)
    client.close()
    print(json.dumps({"config": "C1: %d-word upload+download, %d loopback parties, JSON opens, %s client-party hops"
                                % (a.words, a.parties, a.transport),
                      "upload_ms_median": statistics.median(up), "download_ms_median": statistics.median(down),
                      "reps": a.reps, "note": "fake-Castor tuples generated before each timed call (test dealer, not the path)"}))


if __name__ == "__main__":
    main()
