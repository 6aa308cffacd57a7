"""PCIe ceiling on the GPU box (tool): page-locked HtoD / DtoH copy rates of
large buffers with torch, alone and both directions at once, to price the
host-memory path (bench.py --mode host) against what the link delivers."""
import json
import time

import torch

N = 1 << 30
h = torch.empty(N, dtype=torch.uint8).pin_memory()
h2 = torch.empty(N, dtype=torch.uint8).pin_memory()
d = torch.empty(N, dtype=torch.uint8, device="cuda")
d2 = torch.empty(N, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def rate(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return reps * N / (time.perf_counter() - t0) / 1e9


def both():
    with torch.cuda.stream(s1):
        d.copy_(h, non_blocking=True)
    with torch.cuda.stream(s2):
        h2.copy_(d2, non_blocking=True)


out = {"htod_GBps": rate(lambda: d.copy_(h, non_blocking=True)),
       "dtoh_GBps": rate(lambda: h2.copy_(d2, non_blocking=True)),
       "bidir_GBps_each_way": rate(both)}
print(json.dumps(out))

# caller memory page-locked in place (hipHostRegister, what amph_host_register
# does to a numpy array) instead of hipHostMalloc'd
import os, sys  # noqa: E401,E402
import numpy as np  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import amphora_amd as A  # noqa: E402
from amphora_amd.spdz import TEST_PRIME, TEST_R, TEST_RINV  # noqa: E402
ctx = A.Context(TEST_PRIME, TEST_R, TEST_RINV)
a = np.ones(N, np.uint8)
ctx.host_register(a)
ha = torch.from_numpy(a)
out["registered_is_pinned"] = bool(ha.is_pinned())
out["registered_htod_GBps"] = rate(lambda: d.copy_(ha, non_blocking=True))
half = N // 2


def two_streams():
    with torch.cuda.stream(s1):
        d[:half].copy_(h[:half], non_blocking=True)
    with torch.cuda.stream(s2):
        d[half:].copy_(h[half:], non_blocking=True)


out["htod_two_streams_GBps"] = rate(two_streams)
print(json.dumps(out))
