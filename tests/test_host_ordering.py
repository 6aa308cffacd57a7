"""The host-copy ordering rule of libamphora_hip (kPageableRule, capi.hip):
hipMemcpyAsync only with page-locked host memory; pageable memory moves with
a blocking hipMemcpy once the context stream is idle.

* CPU: a static check of capi.hip -- every hipMemcpyAsync with a host
  operand sits in the batched pipeline (run_batched_impl), whose host
  operands are page-locked (the caller's registered buffer, or the slot's
  pinned staging buffer); device-to-device async copies and stream-ordered
  allocations appear only in device-mode code (the ragged-party tail of
  ragged_odo_call / amph_recombine_object, which stages one word per party
  on the caller's stream).
* GPU: a FRESH process's first calls -- the situation in which round 2 saw
  a pageable async copy arrive after the kernel that read it -- through the
  wire-text K_RV (text staged from pageable memory), the base64 decode with a
  tail (run_tail's copy in) and the exchange decode, each checked against
  Python's base64 / the C oracle.  Run once each; no retry loop.
"""
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CAPI = os.path.join(ROOT, "amphora_amd", "csrc", "capi.hip")


def _function_spans(src: str):
    """(name, start, end) of top-level function bodies (brace matching)."""
    spans = []
    for m in re.finditer(r"^[A-Za-z_][\w:<>,\s\*&]*?\b(\w+)\s*\([^;{]*\)\s*\{", src, re.M):
        depth, i = 0, m.end() - 1
        while i < len(src):
            depth += {"{": 1, "}": -1}.get(src[i], 0)
            if depth == 0:
                break
            i += 1
        spans.append((m.group(1), m.start(), i))
    return spans


def test_async_copies_only_in_the_pinned_pipeline():
    src = open(CAPI).read()
    code = re.sub(r"//[^\n]*", "", src)  # comments may name the call
    spans = _function_spans(code)
    calls = [m for m in re.finditer(r"\bhipMemcpy(?:2D)?Async\s*\(([^;]*)\);", code)]
    assert calls, "expected the batched pipeline's copies"
    device_only = ("stage_tail", "ragged_odo_call", "amph_recombine_object", "amph_party_partner_dev")
    for m in calls:
        owner = [n for n, a, b in spans if a <= m.start() <= b]
        if "hipMemcpyDeviceToDevice" in m.group(1):  # no host operand
            assert owner and owner[-1] in device_only, (m.group(0), owner)
            continue
        assert owner and owner[-1] == "run_batched_impl", \
            "hipMemcpyAsync outside the page-locked pipeline at offset %d (%s)" % (m.start(), owner)
    body = next(code[a:b] for n, a, b in spans if n == "run_batched_impl")
    # host operands: the caller's buffer only when it is page-locked, else the slot's pinned
    # buffer (always for AMPH_F_HOST_IO arrays, which are callbacks, not memory)
    assert "in_pinned[k] = !ins[k].io && amph::is_pinned_host(ins[k].host)" in body
    assert "out_pinned[k] = !outs[k].io && amph::is_pinned_host(outs[k].host)" in body
    # stream-ordered allocation: only the device-mode ragged tail's one-word staging
    for m in re.finditer(r"\bhipMallocAsync\s*\(", code):
        owner = [n for n, a, b in spans if a <= m.start() <= b]
        assert owner and owner[-1] in ("ragged_odo_call", "amph_recombine_object"), owner
        body = next(code[a:b] for n, a, b in spans if n == owner[-1])
        assert "AMPH_F_DEVICE" in body[:body.find("hipMallocAsync")], "device-mode branch only"


_FIRST_CALL = r"""
import base64, sys
import numpy as np
sys.path.insert(0, %(root)r)
import amphora_amd as A
from oracle import amphora_oracle as O
from oracle import coracle
what = sys.argv[1]
ctx = A.Context(O.TEST_PRIME, O.TEST_R, O.TEST_RINV)
F = coracle.test_field(threads=4)
if what == "rv_b64":
    W = 5000
    odos, _ = F.synth_odos(seed=41, n=3, W=W)
    texts = [[base64.b64encode(np.ascontiguousarray(f).tobytes()) for f in o] for o in odos]
    y, ff, bad = ctx.recombine_verify_b64(texts, W)  # the process's first GPU call
    oy, off = F.recombine_verify(odos)
    assert ff == off == -1 and bad == -1 and np.array_equal(y, oy), "first wire-text call"
elif what == "b64_tail":
    raw = np.random.default_rng(5).integers(0, 256, 16 * 1000 + 7, dtype=np.uint8).tobytes()
    text = base64.b64encode(raw)  # padded: the last unit goes through run_tail
    assert ctx.base64_decode(text) == raw, "first base64 decode"
elif what == "xdec":
    mag = np.random.default_rng(6).integers(0, 256, (4096, 2, 16), dtype=np.uint8)
    neg = np.random.default_rng(7).integers(0, 2, (4096, 2), dtype=np.uint8)
    enc = ctx.exchange_encode(mag, neg)  # first call encodes, second decodes the text
    m2, n2 = ctx.exchange_decode(enc, 4096)
    assert np.array_equal(m2, mag) and np.array_equal(n2, neg), "first exchange round trip"
print("ok", what)
"""


@pytest.mark.gpu
@pytest.mark.parametrize("what", ["rv_b64", "b64_tail", "xdec"])
def test_fresh_process_first_call(what):
    script = _FIRST_CALL % {"root": ROOT}
    r = subprocess.run([sys.executable, "-c", script, what], capture_output=True, text=True,
                       timeout=240, cwd=ROOT)
    assert r.returncode == 0 and ("ok " + what) in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])
