"""Parity of the HIP path (libamphora_hip.so via the C ABI) with the CPU
oracle.  Bit-exact: this is integer / byte work.

* golden fixtures (tests/golden, produced by the Python oracle, itself pinned
  to the reference KATs in test_oracle_kat.py) through both the host-pointer
  and the device-pointer (AMPH_F_DEVICE) entry points;
* seeded synthetic inputs at sizes the C oracle (oracle/amphora_oracle.c)
  finishes in seconds, including non-canonical words, faults, ragged sizes,
  every party count 1..5 and 16, and a prime below 2^127;
* BASELINE sizes (C2 1 Mi x 2 parties, C3 16 Mi x 3 parties, and C4 64 Mi x 2
  / C5 256 Mi x 3 whole on one GPU) through
  size-independent properties: verify passes on honest input, the injected
  fault is found at its index, and random word samples match the oracle.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from oracle import amphora_oracle as O  # noqa: E402
from oracle import coracle  # noqa: E402

P, R, RINV = O.TEST_PRIME, O.TEST_R, O.TEST_RINV
NO_FAIL = 0x7F7F7F7F7F7F7F7F


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need a GPU"
    return t


@pytest.fixture(scope="module")
def ctx(torch):
    import amphora_amd as A
    return A.Context(P, R, RINV, device=0)


@pytest.fixture(scope="module")
def F():
    return coracle.test_field(threads=16)


def _cases(golden_dir):
    with open(os.path.join(golden_dir, "manifest.json")) as f:
        return json.load(f)["cases"]


def dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    return t.cpu().numpy()


def ff_dev(t):
    v = int(t.cpu().item())
    return -1 if v == NO_FAIL else v


@pytest.mark.parametrize("idx", range(4))
@pytest.mark.parametrize("mode", ["host", "device"])
def test_golden(golden_dir, ctx, torch, idx, mode):
    case = _cases(golden_dir)[idx]
    d = np.load(os.path.join(golden_dir, case["file"]), allow_pickle=False)
    n = case["parties"]
    on = (lambda a: dev(torch, a)) if mode == "device" else (lambda a: np.ascontiguousarray(a))
    back = host if mode == "device" else (lambda a: a)
    ffv = ff_dev if mode == "device" else (lambda v: v)
    for tag in ("honest", "fault", "noncanon"):
        buf = d["rv_%s_odo" % tag]
        odos = [tuple(on(buf[k, j]) for k in range(5)) for j in range(n)]
        y, ff = ctx.recombine_verify(odos)
        assert ffv(ff) == d["rv_%s_first_fail" % tag][0], tag
        assert np.array_equal(back(y), d["rv_%s_secrets" % tag]), tag
    mo = d["mask_odo"]
    out, ff = ctx.mask_input([tuple(on(mo[k, j]) for k in range(5)) for j in range(n)],
                             on(d["mask_secrets"]))
    assert ffv(ff) == -1 and np.array_equal(back(out), d["mask_out"])
    mf = d["mask_fault_odo"]
    _, ff = ctx.mask_input([tuple(on(mf[k, j]) for k in range(5)) for j in range(n)],
                           on(d["mask_secrets"]))
    assert ffv(ff) == d["mask_fault_first_fail"][0]
    key = int.from_bytes(d["conv_mac_key"].tobytes(), "little")
    for z in (0, 1):
        out = ctx.convert_share(on(d["conv_masked"]), on(d["conv_tuples"]), key, bool(z))
        assert np.array_equal(back(out), d["conv_out_zero%d" % z])
    y, r, v, mag, neg = ctx.odo_pre(on(d["odo_share_data"]), 32, on(d["odo_masks"]),
                                    on(d["odo_triples"]))
    for got, k in ((y, "odo_y"), (r, "odo_r"), (v, "odo_v"), (mag, "odo_diff_mag"),
                   (neg, "odo_diff_neg")):
        assert np.array_equal(back(got), d[k]), k
    mags = [on(d["odo_diff_mag"])] + [on(d["odo_partner_mag"][j]) for j in range(n - 1)]
    negs = [on(d["odo_diff_neg"])] + [on(d["odo_partner_neg"][j]) for j in range(n - 1)]
    assert np.array_equal(back(ctx.open_diffs(mags, negs)), d["odo_opened"])
    for pid in (0, 1):
        w, u = ctx.odo_post(on(d["odo_opened"]), on(d["odo_triples"]), pid == 0)
        assert np.array_equal(back(w), d["odo_w_p%d" % pid])
        assert np.array_equal(back(u), d["odo_u_p%d" % pid])
        # the fused open + post from the parties' diffs gives the same words
        w, u = ctx.open_post(mags, negs, on(d["odo_triples"]), pid == 0)
        assert np.array_equal(back(w), d["odo_w_p%d" % pid])
        assert np.array_equal(back(u), d["odo_u_p%d" % pid])


@pytest.mark.parametrize("n,W", [(1, 777), (2, 100_003), (3, 65_536), (4, 4097), (5, 3000),
                                 (16, 513)])
def test_recombine_verify_vs_c_oracle(ctx, F, n, W):
    odos, _ = F.synth_odos(seed=100 + n, n=n, W=W, noncanon_permille=30)
    y, ff = ctx.recombine_verify(odos)
    oy, off = F.recombine_verify(odos)
    assert ff == off == -1 and np.array_equal(y, oy)
    fault = W // 3
    odos, _ = F.synth_odos(seed=200 + n, n=n, W=W, fault_index=fault)
    y, ff = ctx.recombine_verify(odos)
    oy, off = F.recombine_verify(odos)
    assert ff == off == fault and np.array_equal(y, oy)


@pytest.mark.parametrize("n,W", [(1, 1000), (2, 262_145), (3, 40_000), (6, 999), (16, 4099)])
def test_mask_input_vs_c_oracle(ctx, F, n, W):
    odos, _ = F.synth_odos(seed=300 + n, n=n, W=W, noncanon_permille=10)
    secrets = F.synth_words(seed=7, count=W, mont=False)
    secrets[::7] = 0xFF  # raw 128-bit integers >= p are reduced too
    out, ff = ctx.mask_input(odos, secrets)
    oo, off = F.mask_input(secrets, odos)
    assert ff == off == -1 and np.array_equal(out, oo)


def test_mask_input_fewer_secrets_than_masks(ctx, F):
    odos, _ = F.synth_odos(seed=11, n=2, W=5000, fault_index=4500)
    secrets = F.synth_words(seed=8, count=3000, mont=False)
    out, ff = ctx.mask_input(odos, secrets)
    assert ff == 4500  # the verify covers every mask word
    import torch
    dodos = [tuple(torch.from_numpy(f).cuda() for f in o) for o in odos]
    _, dff = ctx.mask_input(dodos, torch.from_numpy(secrets).cuda())
    assert ff_dev(dff) == 4500  # device path: verify-only tail reports global indices
    odos, _ = F.synth_odos(seed=11, n=2, W=5000)
    out, ff = ctx.mask_input(odos, secrets)
    oo, _ = F.mask_input(secrets, [tuple(f[:3000] for f in o) for o in odos])
    assert ff == -1 and np.array_equal(out, oo)
    dodos = [tuple(torch.from_numpy(f).cuda() for f in o) for o in odos]
    dout, dff = ctx.mask_input(dodos, torch.from_numpy(secrets).cuda())
    assert ff_dev(dff) == -1 and np.array_equal(host(dout), oo)


def _oracle_create_secret(F, odos, secrets):
    """The oracle's createSecret arithmetic (amphora_oracle.py
    create_secret_masked_inputs, DefaultAmphoraClient.java:150-160): which
    exception, if any, the reference raises first."""
    util = O.ClientSecretShareUtil(P, R, RINV)
    oodos = [O.OutputDeliveryObject(*[f.tobytes() for f in o]) for o in odos]
    vals = [int.from_bytes(bytes(w), "little") for w in secrets]
    try:
        O.create_secret_masked_inputs(util, vals, oodos)
    except O.IntegrityVerificationException:
        return "verify"
    except IndexError:
        return "index"
    return "ok"


@pytest.mark.parametrize("fault", [450, -1])
def test_mask_input_more_secrets_than_masks_verifies_first(ctx, F, torch, fault):
    """with more secret words than masks the C ABI
    verifies every mask first and returns AMPH_E_VERIFY (first_fail set) for
    a tampered set, AMPH_E_LEN only for an honest one -- the reference's
    order (verifyOutputDeliveryObjects :153 before inputMasks.get(i) :160),
    checked against the oracle, in host and device mode and through the
    fused wire call."""
    import amphora_amd as A
    W, S = 700, 900
    odos, _ = F.synth_odos(seed=61, n=3, W=W, fault_index=fault)
    secrets = F.synth_words(seed=62, count=S, mont=False)
    want = _oracle_create_secret(F, odos, secrets)
    assert want == ("verify" if fault >= 0 else "index")
    dodos = [tuple(dev(torch, f) for f in o) for o in odos]
    texts = [tuple(ctx.base64_encode(f.tobytes()) for f in o) for o in odos]
    calls = [("host", lambda: ctx.mask_input(odos, secrets), lambda ff: ff),
             ("device", lambda: ctx.mask_input(dodos, dev(torch, secrets)), ff_dev),
             ("b64", lambda: ctx.mask_input_b64(texts, W, secrets, records=True)[2], lambda ff: ff)]
    for mode, call, ffv in calls:
        if want == "verify":
            r = call()
            ff = r[1] if isinstance(r, tuple) else r
            assert ffv(ff) == fault, mode
        else:
            with pytest.raises(A.AmphoraNativeError) as e:
                call()
            assert e.value.status == A._lib.AMPH_E_LEN, mode
    # the client mirror maps the statuses to the reference's exceptions
    from amphora_amd import client as CL
    from amphora_amd.entities import IntegrityVerificationException, OutputDeliveryObject, Secret
    util = CL.SecretShareUtil(ctx)
    sec = Secret.of([], [int.from_bytes(bytes(w), "little") for w in secrets])
    with pytest.raises(IntegrityVerificationException if want == "verify" else IndexError):
        CL.create_masked_input(util, sec, [OutputDeliveryObject(*[f.tobytes() for f in o]) for o in odos])


def test_host_batches_report_global_index(ctx, F):
    odos, _ = F.synth_odos(seed=12, n=3, W=2500, fault_index=1777)
    ctx.set_batch_words(1000)
    try:
        y, ff = ctx.recombine_verify(odos)
        oy, _ = F.recombine_verify(odos)
    finally:
        ctx.set_batch_words(4 << 20)
    assert ff == 1777 and np.array_equal(y, oy)


def test_host_batches_sixteen_parties(ctx, F):
    """AMPH_MAX_PARTIES through the host pipeline: 16 ODOs (80 input streams
    per batch, 81 with the secrets), several batches, a MAC fault in a later
    batch and in the verify-only tail of amph_mask_input, against the oracle."""
    W, S = 9001, 5000
    odos, _ = F.synth_odos(seed=17, n=16, W=W, noncanon_permille=10)
    secrets = F.synth_words(seed=18, count=S, mont=False)
    bad, _ = F.synth_odos(seed=19, n=16, W=W, fault_index=7777)
    ctx.set_batch_words(2048)
    try:
        y, ff = ctx.recombine_verify(odos)
        m, mf = ctx.mask_input(odos, secrets)
        _, bff = ctx.recombine_verify(bad)
        _, bmf = ctx.mask_input(bad, secrets)
    finally:
        ctx.set_batch_words(4 << 20)
    oy, off = F.recombine_verify(odos)
    om, omf = F.mask_input(secrets, [tuple(f[:S] for f in o) for o in odos])
    assert ff == off == -1 and np.array_equal(y, oy)
    assert mf == omf == -1 and np.array_equal(m, om)
    assert bff == bmf == 7777


def test_host_stream_pinned_and_pageable(ctx, F):
    """Many batches through the 3-slot pipeline, pageable and page-locked
    caller buffers mixed (the staging copy is skipped for the latter)."""
    W = 70_001
    odos, buf = F.synth_odos(seed=13, n=2, W=W, fault_index=65_000)
    secrets = F.synth_words(seed=14, count=W, mont=False)
    ctx.set_batch_words(8192)
    try:
        y1, ff1 = ctx.recombine_verify(odos)
        ctx.host_register(buf)
        try:
            y2, ff2 = ctx.recombine_verify(odos)
            m2, mf = ctx.mask_input(odos, secrets)
        finally:
            ctx.host_unregister(buf)
    finally:
        ctx.set_batch_words(4 << 20)
    oy, off = F.recombine_verify(odos)
    om, omf = F.mask_input(secrets, odos)
    assert ff1 == ff2 == off == 65_000 and mf == omf == 65_000
    assert np.array_equal(y1, oy) and np.array_equal(y2, oy) and np.array_equal(m2, om)


def test_host_outputs_reused_and_page_locked(ctx, F):
    """Caller-owned output buffers (out=), page-locked or not, reused across
    calls: batched DtoH straight into them (no staging copy-out)."""
    W = 50_003
    odos, _ = F.synth_odos(seed=15, n=3, W=W)
    secrets = F.synth_words(seed=16, count=W, mont=False)
    oy, off = F.recombine_verify(odos)
    om, omf = F.mask_input(secrets, odos)
    ys = np.zeros((W, 16), np.uint8)
    ms = np.zeros((W, 16), np.uint8)
    ctx.set_batch_words(4096)
    try:
        for pinned in (False, True, True):
            if pinned:
                ctx.host_register(ys)
                ctx.host_register(ms)
            try:
                y, ff = ctx.recombine_verify(odos, out=ys)
                m, mf = ctx.mask_input(odos, secrets, out=ms)
            finally:
                if pinned:
                    ctx.host_unregister(ys)
                    ctx.host_unregister(ms)
            assert y is ys and m is ms and ff == off == -1 and mf == omf == -1
            assert np.array_equal(ys, oy) and np.array_equal(ms, om)
            ys[:] = 0
            ms[:] = 0
    finally:
        ctx.set_batch_words(4 << 20)


def test_concurrent_callers(ctx, F):
    """Host-path calls from several threads (ctypes releases the GIL): one
    shared context (calls serialise on its lock) and a second context of its
    own; every result matches the oracle, faults stay with their caller."""
    import threading
    import amphora_amd as A
    ctx2 = A.Context(P, R, RINV, device=0)
    cases = []
    for t in range(6):
        odos, _ = F.synth_odos(seed=500 + t, n=2 + t % 2, W=20_000 + 777 * t,
                               fault_index=(1000 * t if t % 3 == 0 else -1))
        cases.append((odos, F.recombine_verify(odos)))
    got = [None] * len(cases)

    def work(i):
        c = ctx2 if i % 2 else ctx
        for _ in range(3):
            got[i] = c.recombine_verify(cases[i][0])

    th = [threading.Thread(target=work, args=(i,)) for i in range(len(cases))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for (odos, (oy, off)), (y, ff) in zip(cases, got):
        assert ff == off and np.array_equal(y, oy)


def test_multi_device_context(ctx, F):
    """amph_ctx_create_multi with the one GPU named three times: host-pointer
    calls run as three concurrent shards (each its own batched pipeline) and
    must equal the single-device results, with global first-fail indices."""
    import amphora_amd as A
    g = A.Context(P, R, RINV, devices=[0, 0, 0])
    g.set_batch_words(8192)  # several batches per shard
    W = 100_003  # shards of 33 335 words
    # the shards run on the sub-contexts' long-lived workers, not on threads
    # started per call
    st0 = g.stats()
    assert st0["device_workers"] == 3 and st0["worker_tasks"] == 0
    for fault in (-1, 70_000, 33_334, 33_335):
        odos, _ = F.synth_odos(seed=600, n=3, W=W, fault_index=fault, noncanon_permille=10)
        y, ff = g.recombine_verify(odos)
        oy, off = F.recombine_verify(odos)
        assert ff == off == fault and np.array_equal(y, oy), fault
    st1 = g.stats()
    assert st1["device_workers"] == 3 and st1["worker_tasks"] == 3 * 4
    assert st1["kernel_launches"] >= 3 * 4
    # two faults in different shards: the smaller index wins
    odos, _ = F.synth_odos(seed=601, n=2, W=W, fault_index=90_000)
    odos[1][4][40_000, 0] ^= 1
    assert g.recombine_verify(odos)[1] == 40_000
    # masking with fewer secrets than masks: the verify-only tail is sharded too
    odos, _ = F.synth_odos(seed=602, n=2, W=W, fault_index=95_000)
    secrets = F.synth_words(seed=603, count=60_000, mont=False)
    out, ff = g.mask_input(odos, secrets)
    assert ff == 95_000
    odos, _ = F.synth_odos(seed=602, n=2, W=W)
    out, ff = g.mask_input(odos, secrets)
    oo, _ = F.mask_input(secrets, [tuple(f[:60_000] for f in o) for o in odos])
    assert ff == -1 and np.array_equal(out, oo)
    # other word-parallel calls agree with the single-device context
    words = F.synth_words(seed=604, count=W, mont=True)
    assert np.array_equal(g.from_gfp(words), ctx.from_gfp(words))
    assert np.array_equal(g.to_gfp(words), ctx.to_gfp(words))
    tuples = F.synth_words(seed=605, count=2 * W, mont=True).reshape(W, 32)
    assert np.array_equal(g.convert_share(words, tuples, 12345, False),
                          ctx.convert_share(words, tuples, 12345, False))
    assert np.array_equal(g.base64_encode_words(words), ctx.base64_encode_words(words))
    # fewer words than devices
    odos, _ = F.synth_odos(seed=606, n=2, W=2)
    y, ff = g.recombine_verify(odos)
    assert ff == -1 and np.array_equal(y, F.recombine_verify(odos)[0])


def test_empty_and_single(ctx):
    z = np.zeros((0, 16), np.uint8)
    y, ff = ctx.recombine_verify([(z,) * 5, (z,) * 5])
    assert y.shape == (0, 16) and ff == -1
    assert ctx.recombine([z, z]).shape == (0, 16)
    out = ctx.convert_share(z, np.zeros((0, 32), np.uint8), 5, False)
    assert out.shape == (0, 32)


def test_party_kernels_vs_c_oracle(ctx, F):
    W = 50_001
    masked = F.synth_words(seed=21, count=W)
    tuples = F.synth_words(seed=22, count=2 * W).reshape(W, 32)
    key = 123456789123456789123456789 % P
    for z in (False, True):
        assert np.array_equal(ctx.convert_share(masked, tuples, key, z),
                              F.convert_share(masked, tuples, key, z))
    share = ctx.convert_share(masked, tuples, key, False)
    masks = F.synth_words(seed=23, count=4 * W).reshape(2 * W, 32)
    triples = F.synth_words(seed=24, count=12 * W).reshape(2 * W, 96)
    for stride, data in ((32, share), (16, masked)):
        got = ctx.odo_pre(data, stride, masks, triples)
        exp = F.odo_pre(data, stride, masks, triples)
        for g, e in zip(got, exp):
            assert np.array_equal(g, e)
    _, _, _, mag, neg = got
    pm = F.synth_words(seed=25, count=4 * W).reshape(2 * W, 2, 16)
    pn = (F.synth_words(seed=26, count=W)[:, :4].reshape(2 * W, 2) & 1).astype(np.uint8)
    opened = ctx.open_diffs([mag, pm], [neg, pn])
    assert np.array_equal(opened, F.recombine_diffs([mag, pm], [neg, pn]))
    for p0 in (True, False):
        w, u = ctx.odo_post(opened, triples, p0)
        ew, eu = F.odo_post(opened, triples, p0)
        assert np.array_equal(w, ew) and np.array_equal(u, eu)
        w, u = ctx.open_post([mag, pm], [neg, pn], triples, p0)
        assert np.array_equal(w, ew) and np.array_equal(u, eu)


@pytest.mark.parametrize("n,W", [(1, 1), (2, 64), (2, 100_003), (3, 65_537), (4, 4097), (5, 3000),
                                 (16, 513)])
def test_open_post_vs_c_oracle(ctx, F, n, W):
    """amph_open_post (recombineDiffs + multiplySharedSecrets fused) against
    the C oracle's recombine_diffs + odo_post, every party count path (1-4
    templated, more at run time), ragged tails of the 128-pair workgroups,
    sign bytes other than 0/1 (any nonzero byte is negative), host and
    device buffers."""
    import torch
    triples = F.synth_words(seed=40 + n, count=12 * W).reshape(2 * W, 96)
    mags = [F.synth_words(seed=50 + j, count=4 * W).reshape(2 * W, 2, 16) for j in range(n)]
    negs = [(F.synth_words(seed=70 + j, count=W)[:, :4].reshape(2 * W, 2) % 3).astype(np.uint8)
            for j in range(n)]
    opened = F.recombine_diffs(mags, negs)
    for p0 in (True, False):
        ew, eu = F.odo_post(opened, triples, p0)
        w, u = ctx.open_post(mags, negs, triples, p0)
        assert np.array_equal(w, ew) and np.array_equal(u, eu), p0
        dw, du = ctx.open_post([torch.from_numpy(m).cuda() for m in mags],
                               [torch.from_numpy(x).cuda() for x in negs],
                               torch.from_numpy(triples).cuda(), p0)
        torch.cuda.synchronize()
        assert np.array_equal(dw.cpu().numpy(), ew) and np.array_equal(du.cpu().numpy(), eu), p0


def test_open_post_host_batches(ctx, F):
    """Host-pointer open_post through the batched 3-slot pipeline."""
    W = 20_011
    triples = F.synth_words(seed=91, count=12 * W).reshape(2 * W, 96)
    mags = [F.synth_words(seed=92 + j, count=4 * W).reshape(2 * W, 2, 16) for j in range(3)]
    negs = [(F.synth_words(seed=95 + j, count=W)[:, :4].reshape(2 * W, 2) & 1).astype(np.uint8)
            for j in range(3)]
    ew, eu = F.odo_post(F.recombine_diffs(mags, negs), triples, False)
    ctx.set_batch_words(4096)
    try:
        w, u = ctx.open_post(mags, negs, triples, False)
    finally:
        ctx.set_batch_words(4 << 20)
    assert np.array_equal(w, ew) and np.array_equal(u, eu)


def test_codec_and_mask_words(ctx, F):
    W = 10_000
    x = F.synth_words(seed=31, count=W, mont=False)
    x[::5] = 0xFF
    g = ctx.to_gfp(x)
    spdz = O.MpSpdzIntegrationUtils(P, R, RINV)
    xs = [int.from_bytes(w.tobytes(), "little") for w in x[:500]]
    assert [bytes(w) for w in g[:500]] == [spdz.to_gfp(v) for v in xs]
    back = ctx.from_gfp(g)
    assert [int.from_bytes(w.tobytes(), "little") for w in back[:500]] == [v % P for v in xs]
    m = F.synth_words(seed=32, count=W, mont=False)
    mw = ctx.mask_words(x, m)
    ms = [int.from_bytes(w.tobytes(), "little") for w in m[:500]]
    assert [bytes(w) for w in mw[:500]] == [spdz.to_gfp((a - b) % P) for a, b in zip(xs, ms)]


def test_small_prime_path(torch, F):
    """p = 2^89 - 1 < 2^127: the !BIG canonicalisation path."""
    import amphora_amd as A
    p = 2 ** 89 - 1
    r = pow(2, 128, p)
    rinv = pow(r, -1, p)
    c = A.Context(p, r, rinv)
    Fs = coracle.Field(p, r, rinv, threads=16)
    odos, _ = Fs.synth_odos(seed=41, n=3, W=20_000, fault_index=12_345)
    # raw words may be any 128-bit value: scramble some above p
    odos[0][0][::3, 15] = 0xEE
    y, ff = c.recombine_verify(odos)
    oy, off = Fs.recombine_verify(odos)
    assert ff == off and np.array_equal(y, oy)
    secrets = Fs.synth_words(seed=42, count=20_000, mont=False)
    odos, _ = Fs.synth_odos(seed=43, n=2, W=20_000)
    out, ff = c.mask_input(odos, secrets)
    oo, off = Fs.mask_input(secrets, odos)
    assert ff == off == -1 and np.array_equal(out, oo)


def test_device_synth_is_honest(ctx, F, torch):
    odos, buf, plain = ctx.synth_odos(seed=5, n=3, words=30_000, noncanon_permille=20,
                                      with_plain=True)
    torch.cuda.synchronize()
    hodos = [tuple(host(f) for f in o) for o in odos]
    oy, off = F.recombine_verify(hodos)
    assert off == -1 and np.array_equal(oy, host(plain))
    odos, _, _ = ctx.synth_odos(seed=5, n=2, words=30_000, fault_index=29_999)
    _, off = F.recombine_verify([tuple(host(f) for f in o) for o in odos])
    assert off == 29_999


def _sample_check(F, odos_dev, y_dev, idx, host_fn):
    sub = [tuple(host_fn(f[idx]) for f in o) for o in odos_dev]
    oy, off = F.recombine_verify(sub)
    assert off == -1
    assert np.array_equal(host_fn(y_dev[idx]), oy)


@pytest.mark.parametrize("n,W", [(2, 1 << 20), (3, 1 << 24), (2, 1 << 26), (3, 1 << 28)])
def test_baseline_sizes(ctx, F, torch, n, W):
    """C2 (1 Mi words, 2 parties), C3 (16 Mi words, 3 parties), and the whole
    of C4 (64 Mi x 2) and C5 (256 Mi x 3, 60 GiB of shares: byte offsets far
    past 2^32) resident on ONE GPU -- the maximum sizes BASELINE names."""
    odos, buf, _ = ctx.synth_odos(seed=99, n=n, words=W, noncanon_permille=5)
    y, ff = ctx.recombine_verify(odos)
    assert ff_dev(ff) == -1
    idx = torch.randint(0, W, (4096,), device="cuda", generator=torch.Generator("cuda").manual_seed(1))
    _sample_check(F, odos, y, idx, host)
    secrets = ctx.synth_words(seed=98, count=W)
    masked, ff = ctx.mask_input(odos, secrets)
    assert ff_dev(ff) == -1
    # round trip (DefaultAmphoraClientTest.java:193-235): masked + mask == secret
    sub_o = [tuple(host(f[idx]) for f in o) for o in odos]
    sec = host(secrets[idx])
    oo, _ = F.mask_input(sec, sub_o)
    assert np.array_equal(host(masked[idx]), oo)
    del buf, odos, y, secrets, masked
    torch.cuda.empty_cache()
    # faulted: the kernel finds exactly the injected index
    fault = W // 3
    odos, buf, _ = ctx.synth_odos(seed=97, n=n, words=W, fault_index=fault)
    _, ff = ctx.recombine_verify(odos)
    assert ff_dev(ff) == fault
    del buf
    torch.cuda.empty_cache()


def test_timing_events_stamp_the_next_launch(ctx, F, torch):
    """amph_time_next_launch with amph_timing_event_create events (what
    bench.py uses): the events time exactly the next kernel launch of an
    amph_* call, a positive duration far below the wall time of a
    synchronising call, and the launch's results are unaffected."""
    import amphora_amd as A
    W, n = 1 << 20, 2
    odos, _, _ = ctx.synth_odos(seed=5, n=n, words=W)
    y0, ff0 = ctx.recombine_verify(odos)
    torch.cuda.synchronize()
    e0, e1 = A._lib.TimingEvent(), A._lib.TimingEvent()
    assert A._lib.lib.amph_time_next_launch(e0.handle, e1.handle) == 0
    y1, ff1 = ctx.recombine_verify(odos)
    torch.cuda.synchronize()
    ms = e0.elapsed_ms(e1)
    assert 0.0 < ms < 50.0
    assert int(ff0.item()) == int(ff1.item()) == A._lib.AMPH_NO_FAILURE
    assert torch.equal(y0, y1)
    # the same call bracketed by events recorded on its stream
    import ctypes as C
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert A._lib.lib.amph_timing_event_record(e0.handle, s) == 0
    ctx.recombine_verify(odos)
    assert A._lib.lib.amph_timing_event_record(e1.handle, s) == 0
    torch.cuda.synchronize()
    assert 0.0 < e0.elapsed_ms(e1) < 50.0


def test_device_arrays_must_be_aligned(ctx, torch):
    """Device-pointer word arrays are moved as 16-byte vectors: a misaligned
    one is rejected with AMPH_E_PARAM before any launch, an aligned view of
    the same storage works."""
    import amphora_amd as A
    W = 1000
    raw = torch.zeros(5 * 2 * W * 16 + 64, dtype=torch.uint8, device="cuda")
    odd = raw[8:8 + 5 * 2 * W * 16].view(5, 2, W, 16)   # 8-byte aligned only
    even = raw[16:16 + 5 * 2 * W * 16].view(5, 2, W, 16)
    for buf, ok in ((odd, False), (even, True)):
        odos = [tuple(buf[k, j] for k in range(5)) for j in range(2)]
        if ok:
            y, ff = ctx.recombine_verify(odos)
            torch.cuda.synchronize()
            assert y.shape == (W, 16)
        else:
            with pytest.raises(A._lib.AmphoraNativeError, match="16-byte aligned"):
                ctx.recombine_verify(odos)
    secrets = raw[24:24 + 16 * W].view(W, 16)
    with pytest.raises(A._lib.AmphoraNativeError, match="16-byte aligned"):
        ctx.to_gfp(secrets)
    with pytest.raises(A._lib.AmphoraNativeError, match="16-byte aligned"):
        ctx.base64_encode_words(secrets)
    rec = raw[4:4 + 24 * 100].view(100, 24)  # 4-byte aligned records
    with pytest.raises((A._lib.AmphoraNativeError, ValueError), match="8-byte aligned"):
        ctx.base64_decode_words(rec)


def test_stream_probe_pattern(ctx, F):
    """amph_stream_probe (bench.py's same-pattern ceiling kernel) reads every
    array K_MASK reads: its output is the XOR of all of them."""
    import ctypes as C
    import torch
    import amphora_amd as A
    for n in (2, 3, 6):
        W = 10_007
        odos, _ = F.synth_odos(seed=300 + n, n=n, W=W)
        sec = F.synth_words(seed=310 + n, count=W)
        dodos = [tuple(torch.from_numpy(f).cuda() for f in o) for o in odos]
        arr, _ = ctx._odo_structs(dodos)
        ds = torch.from_numpy(sec).cuda()
        out = torch.empty((W, 16), dtype=torch.uint8, device="cuda")
        stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
        assert A._lib.lib.amph_stream_probe(ctx._h, arr, n, ds.data_ptr(), W, out.data_ptr(), stream) == 0
        exp = sec.copy()
        for o in odos:
            for f in o:
                exp ^= f
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), exp), n


def test_host_verdicts_follow_the_kernels(ctx, F):
    """Host-pointer calls whose only result is the verdict (amph_verify; the
    verify-only tail of amph_mask_input) report a fault in the LAST words of
    the last batch every time: the verdict is read only after the kernels."""
    W = 200_003
    odos, _ = F.synth_odos(seed=1300, n=2, W=W, fault_index=W - 1)
    secrets = F.synth_words(seed=1301, count=1000, mont=False)
    y, r, v, w, u = (np.ascontiguousarray(F.recombine([o[k] for o in odos])) for k in range(5))
    ctx.set_batch_words(65_536)
    try:
        for _ in range(12):
            assert ctx.verify(y, r, u, v, w) == W - 1
            assert ctx.mask_input(odos, secrets)[1] == W - 1
    finally:
        ctx.set_batch_words(4 << 20)


def test_small_calls_back_to_back_same_addresses(ctx, F):
    """the small-call arena (run_small) is read and written in
    place by the kernels at the same addresses on every call; many calls in
    a row with different inputs must each see their own inputs (the arena is
    fine-grained / coherent host memory, so no line cached by an earlier
    call is served).  Every result is compared with the oracle."""
    W = 500  # well under AMPH_SMALL_BYTES: every call takes the small path
    for i in range(60):
        odos, _ = F.synth_odos(seed=7000 + i, n=2, W=W, fault_index=(i * 37) % W if i % 3 == 0 else -1)
        secrets = F.synth_words(seed=8000 + i, count=W, mont=False)
        y, ff = ctx.recombine_verify(odos)
        oy, off = F.recombine_verify(odos)
        assert ff == off and np.array_equal(y, oy), i
        m, mf = ctx.mask_input(odos, secrets)
        om, omf = F.mask_input(secrets, odos)
        assert mf == omf and np.array_equal(m, om), i
