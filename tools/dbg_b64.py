import base64, sys, numpy as np
sys.path.insert(0, '.')
import amphora_amd as A
from oracle import amphora_oracle as O
from oracle import coracle
F = coracle.test_field(threads=8)
ctx = A.Context(O.TEST_PRIME, O.TEST_R, O.TEST_RINV)
for (W, stride) in [(777, 32), (64, 32), (65, 32), (128, 32), (5000, 16)]:
    n = 2
    share = F.synth_words(seed=100, count=W * stride // 16).reshape(W, stride)
    masks = F.synth_words(seed=200, count=4 * W).reshape(2 * W, 32)
    tri = F.synth_words(seed=300, count=12 * W).reshape(2 * W, 96)
    pre = F.odo_pre(share, stride, masks, tri)
    s = ctx.party_begin(share, stride, masks, tri, n)
    s.partner(1, s.text())
    got = s.finish_b64(True)
    for k in range(3):
        want = base64.b64encode(pre[k].tobytes())
        g = got[k]
        if g != want:
            d = next(i for i in range(len(want)) if g[i] != want[i])
            print("W", W, "stride", stride, "field", k, "first diff at char", d, "unit", d // 16, "word", (d // 16) * 12 // 16, g[d-8:d+24], want[d-8:d+24])
        else:
            print("W", W, "stride", stride, "field", k, "ok")
    s.close()
