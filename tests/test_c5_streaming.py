"""BASELINE config C5 at its size: 256 Mi words x 3 parties streamed from
page-locked host memory through the GPU in 4 Mi-word batches (the 3-slot
HtoD / kernel / DtoH pipeline of run_batched, capi.hip), through the two
host-pointer calls the client makes -- createSecret's verify + mask
(amph_mask_input, DefaultAmphoraClient.java:150-160) and getSecret's
recombine + verify (amph_recombine_verify, :206-217,476-505).

Checks (size-independent): honest verdicts; every canonical
secret equals the one the ODOs were generated from; a 4096-word sample of
both outputs equals the C oracle on the same words; a MAC fault injected at
W // 3 is reported at exactly that index by both calls.  On a box with more
than one GPU the same arrays go through one amph_ctx_create_multi context
over the distinct devices (each streams its contiguous shard over its own
link) and must give the same outputs and the same fault index.

Host memory: one 3-party ODO set (60 GiB) serves as both the mask and the
share ODOs, plus 3 x 4 GiB of secrets / outputs -- 72 GiB page-locked.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from oracle import amphora_oracle as O  # noqa: E402
from oracle import coracle  # noqa: E402

W = 1 << 28          # 256 Mi words
N = 3
BATCH = 1 << 22      # 4 Mi words
SAMPLE = 4096


def _device_count():
    import torch
    return torch.cuda.device_count()


@pytest.fixture(scope="module")
def c5():
    import torch
    import amphora_amd as A
    ctx = A.Context(O.TEST_PRIME, O.TEST_R, O.TEST_RINV, device=0)
    ctx.set_batch_words(BATCH)
    odos_h = np.empty((5, N, W, 16), np.uint8)
    sec_h = np.empty((W, 16), np.uint8)
    plain_h = np.empty((W, 16), np.uint8)
    masked_h = np.empty((W, 16), np.uint8)
    ys_h = np.empty((W, 16), np.uint8)
    arrays = (odos_h, sec_h, plain_h, masked_h, ys_h)
    for a in arrays:
        ctx.host_register(a)  # page-locked: every batch is DMA'd straight from / to it
    try:
        _, buf, plain = ctx.synth_odos(seed=55, n=N, words=W, noncanon_permille=2, with_plain=True)
        torch.from_numpy(odos_h).copy_(buf)
        torch.from_numpy(plain_h).copy_(plain)
        del buf, plain
        torch.from_numpy(sec_h).copy_(ctx.synth_words(seed=56, count=W))
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        odos = [tuple(odos_h[k, j] for k in range(5)) for j in range(N)]
        yield ctx, odos, sec_h, plain_h, masked_h, ys_h
    finally:
        for a in arrays:
            ctx.host_unregister(a)


def _sample_check(odos, sec_h, masked_h, ys_h):
    F = coracle.test_field(threads=8)
    idx = np.unique(np.random.default_rng(9).integers(0, W, SAMPLE))
    idx = np.concatenate([idx, [0, BATCH - 1, BATCH, W - 1]])
    so = [tuple(np.ascontiguousarray(f[idx]) for f in o) for o in odos]
    exp_m, f1 = F.mask_input(np.ascontiguousarray(sec_h[idx]), so)
    exp_y, f2 = F.recombine_verify(so)
    assert f1 == f2 == -1
    assert np.array_equal(masked_h[idx], exp_m), "masked words differ from the oracle"
    assert np.array_equal(ys_h[idx], exp_y), "canonical secrets differ from the oracle"


def test_c5_streamed_256Mi_x3(c5):
    ctx, odos, sec_h, plain_h, masked_h, ys_h = c5
    masked_h.fill(0)
    ys_h.fill(0)
    _, ff = ctx.mask_input(odos, sec_h, out=masked_h)
    assert ff == -1
    _, ff = ctx.recombine_verify(odos, out=ys_h)
    assert ff == -1
    assert np.array_equal(ys_h, plain_h), "canonical secrets != the generated ones"
    _sample_check(odos, sec_h, masked_h, ys_h)
    fault = W // 3
    odos[1][3][fault, 0] ^= 1  # party 1's w share of word W // 3
    try:
        assert ctx.recombine_verify(odos, out=ys_h)[1] == fault
        assert ctx.mask_input(odos, sec_h, out=masked_h)[1] == fault
    finally:
        odos[1][3][fault, 0] ^= 1


@pytest.mark.skipif(_device_count() < 2, reason="one GPU visible: amph_ctx_create_multi needs distinct devices")
def test_c5_multi_device_context(c5):
    import amphora_amd as A
    ctx, odos, sec_h, plain_h, masked_h, ys_h = c5
    devs = list(range(min(_device_count(), 8)))
    multi = A.Context(O.TEST_PRIME, O.TEST_R, O.TEST_RINV, devices=devs)
    multi.set_batch_words(BATCH)
    ys_h.fill(0)
    assert multi.recombine_verify(odos, out=ys_h)[1] == -1
    assert np.array_equal(ys_h, plain_h)
    masked_h.fill(0)
    assert multi.mask_input(odos, sec_h, out=masked_h)[1] == -1
    _sample_check(odos, sec_h, masked_h, ys_h)
    fault = W // 3
    odos[1][3][fault, 0] ^= 1
    try:
        assert multi.recombine_verify(odos, out=ys_h)[1] == fault
    finally:
        odos[1][3][fault, 0] ^= 1
