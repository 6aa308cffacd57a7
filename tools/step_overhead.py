"""Where does a bench step's time go beyond the two kernels? (tool)

Times 200 steps of K_MASK + K_RV at C2 four ways in one process:
  events  - amph_time_next_launch events (torch, default flags) on every launch
  nofence - the same with amph_timing_event_create events (no system fence)
  *_5th   - events on every 5th step only
  plain   - no events
  graph   - 20 steps captured in one torch.cuda.CUDAGraph, replayed
  kernels - sum of the per-kernel event durations (the floor)
"""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import amphora_amd as A  # noqa: E402
from amphora_amd.spdz import TEST_PRIME, TEST_R, TEST_RINV  # noqa: E402

W, n, STEPS = 1 << 20, 2, 200
ctx = A.Context(TEST_PRIME, TEST_R, TEST_RINV)
mo, mb, _ = ctx.synth_odos(seed=1, n=n, words=W)
so, sb, _ = ctx.synth_odos(seed=2, n=n, words=W)
sec = ctx.synth_words(seed=3, count=W)
marr, _ = ctx._odo_structs(mo)
sarr, _ = ctx._odo_structs(so)
masked = torch.empty((W, 16), dtype=torch.uint8, device="cuda")
ys = torch.empty((W, 16), dtype=torch.uint8, device="cuda")
ff = torch.full((2,), A._lib.AMPH_NO_FAILURE, dtype=torch.int64, device="cuda")
ffp = [C.cast(C.c_void_p(ff.data_ptr() + 8 * i), C.POINTER(C.c_int64)) for i in range(2)]
flags = A._lib.AMPH_F_DEVICE | A._lib.AMPH_F_ACCUMULATE
L = A._lib.lib


def step(stream, ev=None):
    if ev:
        L.amph_time_next_launch(ev[0].cuda_event, ev[1].cuda_event)
    L.amph_mask_input(ctx._h, marr, n, sec.data_ptr(), W, masked.data_ptr(), ffp[0], flags, stream)
    if ev:
        L.amph_time_next_launch(ev[2].cuda_event, ev[3].cuda_event)
    L.amph_recombine_verify(ctx._h, sarr, n, ys.data_ptr(), ffp[1], flags, stream)


def timed(fn, reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn(reps)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


out = {}
stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
for _ in range(10):
    step(stream)
evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(STEPS)]
for e in evs:
    for x in e:
        x.record()
torch.cuda.synchronize()


def run_events(reps):
    for i in range(reps):
        step(stream, evs[i])


out["events_us_per_step"] = timed(run_events, STEPS)
out["kernels_us_per_step"] = sum(e[0].elapsed_time(e[1]) + e[2].elapsed_time(e[3]) for e in evs) / STEPS * 1e3
nf = [[A._lib.TimingEvent() for _ in range(4)] for _ in range(STEPS)]


class _H:  # amph_time_next_launch takes the raw hipEvent_t
    def __init__(self, e):
        self.cuda_event = e.handle


nfh = [[_H(e) for e in q] for q in nf]


def run_nofence(reps, every=1):
    for i in range(reps):
        step(stream, nfh[i] if i % every == 0 else None)


out["nofence_us_per_step"] = timed(run_nofence, STEPS)
out["nofence_kernels_us_per_step"] = sum(q[0].elapsed_ms(q[1]) + q[2].elapsed_ms(q[3])
                                         for q in nf) / STEPS * 1e3
out["events_5th_us_per_step"] = timed(lambda r: [step(stream, evs[i] if i % 5 == 0 else None)
                                                 for i in range(r)], STEPS)
out["nofence_5th_us_per_step"] = timed(lambda r: run_nofence(r, 5), STEPS)
out["plain_us_per_step"] = timed(lambda r: [step(stream) for _ in range(r)], STEPS)
# launch-only CPU cost (no sync): how long does issuing 200 steps take on the host?
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(STEPS):
    step(stream)
out["host_issue_us_per_step"] = (time.perf_counter() - t0) / STEPS * 1e6
torch.cuda.synchronize()
# graph capture on a side stream
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    cs = C.c_void_p(s.cuda_stream)
    step(cs)
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        for _ in range(20):
            step(C.c_void_p(torch.cuda.current_stream().cuda_stream))
torch.cuda.synchronize()
g.replay()
out["graph_us_per_step"] = timed(lambda r: [g.replay() for _ in range(r // 20)], STEPS)
out["verified"] = bool((ff == A._lib.AMPH_NO_FAILURE).all().item())
print(json.dumps(out))
