"""Pinned vs region-copied JNI calls, through the mock
JNIEnv (tests/jni_mock: Java arrays are plain malloc'd memory, as pageable as
a JVM heap; GetByteArrayRegion is a memcpy, as in HotSpot).

    python tools/bench_jni_regions.py [--words 4194304] [--parties 3] [--reps 5]

For the client's recombineVerify and maskInput (host-pointer calls through
the 3-slot pipeline) at W words x N parties, times the JNI entry point with
AMPH_JNI_REGION_BYTES set so the call pins its arrays (the round-3 layer:
GetPrimitiveArrayCritical across the whole GPU call) and so it hands
libamphora_hip region-copy callbacks (AMPH_F_HOST_IO: nothing pinned while
the GPU works).  Prints one JSON line: best-of-reps ms per call each way,
the pins and region copies the mock counted, and the bit-exact check of the
two outputs against each other and the oracle (sampled)."""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--words", type=int, default=4 << 20)
    ap.add_argument("--parties", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import numpy as np
    import amphora_amd  # noqa: F401  (torch's HIP runtime first, as in the tests)
    from oracle import coracle
    from oracle import amphora_oracle as O
    from test_jni_core import CLIENT, Env, le16
    L = C.CDLL(os.path.join(ROOT, "tests", "jni_mock", "libjni_mock.so"))
    vp = C.c_void_p
    L.mock_env.restype = vp
    for f in ("mock_bytes", "mock_objects"):
        getattr(L, f).restype = vp
    L.mock_bytes.argtypes = [C.c_char_p, C.c_int32]
    L.mock_objects.argtypes = [C.POINTER(vp), C.c_int32]
    L.mock_len.argtypes = [vp]
    L.mock_data.restype = vp
    L.mock_data.argtypes = [vp]
    L.mock_exception_class.restype = L.mock_exception_message.restype = C.c_char_p
    L.mock_region_copies.restype = C.c_long
    e = Env(L)
    h = e.call(CLIENT + "ctxCreate", C.c_int64, e.bytes(le16(O.TEST_PRIME)), e.bytes(le16(O.TEST_R)),
               e.bytes(le16(O.TEST_RINV)), None)
    assert h and e.exception() is None
    ctx = C.c_int64(h)
    F = coracle.test_field(threads=8)
    W, n = a.words, a.parties
    odos, _ = F.synth_odos(seed=9, n=n, W=W)
    secrets = F.synth_words(seed=10, count=W, mont=False)
    lists = e.odo_lists(odos)
    sec = e.bytes(secrets)
    res = {"words": W, "parties": n, "reps": a.reps,
           "bytes_per_call": {"recombineVerify": (80 * n + 16) * W, "maskInput": (80 * n + 32) * W}}
    outs = {}
    for mode, thr in (("pinned", str(1 << 62)), ("regions", "0")):
        os.environ["AMPH_JNI_REGION_BYTES"] = thr
        for name in ("recombineVerify", "maskInput"):
            out = e.zeros(16 * W)
            args = (list(lists) + [out]) if name == "recombineVerify" else (list(lists) + [sec, out])
            best = 1e9
            L.mock_clear()
            for _ in range(a.reps):
                t0 = time.perf_counter()
                rc = e.call(CLIENT + name, C.c_int64, ctx, *args)
                best = min(best, time.perf_counter() - t0)
                assert rc == -1 and e.exception() is None, (name, mode, e.exception())
            outs[(mode, name)] = e.read(out)
            res.setdefault(mode, {})[name] = {
                "ms": round(best * 1e3, 2), "GBps": round(res["bytes_per_call"][name] / best / 1e9, 1),
                "pins": L.mock_pins(), "region_copies": L.mock_region_copies()}
    ok = all(outs[("pinned", k)] == outs[("regions", k)] for k in ("recombineVerify", "maskInput"))
    idx = np.random.default_rng(1).integers(0, W, 256)
    oy, _ = F.recombine_verify([tuple(f[idx] for f in o) for o in odos])
    got = np.frombuffer(outs[("regions", "recombineVerify")], np.uint8).reshape(W, 16)[idx]
    res["bit_exact"] = bool(ok and np.array_equal(got, oy))
    e.call(CLIENT + "ctxDestroy", None, ctx)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
