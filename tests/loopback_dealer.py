"""Fake Castor tuple dealer for the loopback harness (TEST INFRASTRUCTURE).

Produces consistent, MAC'd N-party shares of Input Masks and Multiplication
Triples (castor-common 0.2.0 byte layouts: value||mac per share; a triple is
three shares) with Python ints, one stream per party, cached per
(requestId, tupleType) so every party receives its share of the same tuples
-- what Castor guarantees across VCPs.
"""
import random
import threading


INPUT_MASK_GFP = "INPUT_MASK_GFP"
MULTIPLICATION_TRIPLE_GFP = "MULTIPLICATION_TRIPLE_GFP"


class FakeCastor:
    def __init__(self, prime, r, r_inv, mac_keys, seed=0):
        self.p, self.r = prime, r
        self.mac_keys = list(mac_keys)
        self.alpha = sum(mac_keys) % prime
        self.n = len(mac_keys)
        self.rng = random.Random(seed)
        self.cache = {}
        self.calls = []
        self._lock = threading.Lock()  # parties call concurrently

    def to_gfp(self, x):
        """Castor's wire word: Montgomery form x*r mod p, 16 bytes little-endian
        (the assumed mp-spdz-integration encoding)."""
        return (x * self.r % self.p).to_bytes(16, "little")

    def _share(self, x):
        sh = [self.rng.randrange(self.p) for _ in range(self.n - 1)]
        sh.append((x - sum(sh)) % self.p)
        return sh

    def _auth_share(self, x):
        """value and MAC shares of x (sum of MACs = alpha * x)."""
        return list(zip(self._share(x), self._share(self.alpha * x % self.p)))

    def __call__(self, player, request_id, ttype, count):
        with self._lock:
            return self._get(player, request_id, ttype, count)

    def _get(self, player, request_id, ttype, count):
        self.calls.append((player, request_id, ttype, count))
        key = (request_id, ttype)
        if key not in self.cache:
            streams = [bytearray() for _ in range(self.n)]
            g = self.to_gfp
            for _ in range(count):
                if ttype == INPUT_MASK_GFP:
                    parts = [self._auth_share(self.rng.randrange(self.p))]
                else:
                    a, b = self.rng.randrange(self.p), self.rng.randrange(self.p)
                    parts = [self._auth_share(a), self._auth_share(b), self._auth_share(a * b % self.p)]
                for j in range(self.n):
                    for sh in parts:
                        streams[j] += g(sh[j][0]) + g(sh[j][1])
            self.cache[key] = (count, [bytes(s) for s in streams])
        cnt, streams = self.cache[key]
        assert cnt == count, "tuple count mismatch for %s" % (key,)
        return streams[player]
