"""Pin the CPU oracle against the reference's own known-answer tests and
round-trip properties (CPU only; no GPU, no HIP library).

* KAT-1  amphora-service/.../calculation/SecretShareUtilTest.java:68-107
* KAT-2  amphora-service/.../calculation/OutputDeliveryServiceTest.java:55-175,285-382
* KAT-3  amphora-java-client/.../SecretShareUtilTest.java:30-85 (verify pass / fail)
* round trips  amphora-java-client/.../DefaultAmphoraClientTest.java:193-271
"""
import json
import os
import random
import uuid

import numpy as np
import pytest

from oracle import amphora_oracle as O
from oracle import coracle

P, R, RINV = O.TEST_PRIME, O.TEST_R, O.TEST_RINV


@pytest.fixture(scope="module")
def kat(golden_dir):
    with open(os.path.join(golden_dir, "kat.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def spdz():
    return O.MpSpdzIntegrationUtils.of(P, R, RINV)


def test_field_constants(kat):
    assert int(kat["field"]["prime"]) == P
    assert pow(2, 128, P) == R and (R * RINV) % P == 1


def test_encoding_anchors(kat, spdz):
    a = kat["encoding_anchors"]
    assert spdz.to_gfp(1).hex() == a["toGfp(1)"] == "ffffcbdbb5aa28e479c9de70baf8766a"
    assert spdz.to_gfp(90).hex() == a["toGfp(90)"]
    for x in (0, 1, 90, P - 1, 2 ** 127):
        assert spdz.from_gfp(spdz.to_gfp(x)) == x % P


def test_kat1_convert_to_secret_share(kat, spdz):
    k = kat["kat1"]
    mac_key = int(k["mac_key"]) % P
    masked = [spdz.to_gfp(int(x) % P) for x in k["masked_inputs"]]
    masks = [(spdz.to_gfp(int(v) % P), spdz.to_gfp(int(m) % P)) for v, m in k["input_masks"]]
    out = O.convert_to_secret_share(spdz, masked, str(mac_key), masks, k["use_zero_input_as_data"])
    expected = b"".join(spdz.to_gfp(int(x) % P) for x in k["expected_share_words"])
    assert out == expected


def test_kat1_length_mismatch(spdz):
    # SecretShareUtilTest.java:48-66
    with pytest.raises(O.IllegalArgumentException,
                       match="^Received more input data than available inputMasks.$"):
        O.convert_to_secret_share(spdz, [bytes(16)], "", [], False)


def _kat2_streams(k, spdz):
    share_data = b"".join(spdz.to_gfp(v) + spdz.to_gfp(0) for v in k["secret_values"])
    masks = b"".join(spdz.to_gfp(v) + spdz.to_gfp(0) for v in k["input_mask_values"])
    triples = b"".join(spdz.to_gfp(a) + spdz.to_gfp(0) + spdz.to_gfp(b) + spdz.to_gfp(0)
                       + spdz.to_gfp(c) + spdz.to_gfp(0) for a, b, c in k["triples"])
    return share_data, masks, triples


def test_kat2_output_delivery(kat, spdz):
    k = kat["kat2"]
    share_data, masks, triples = _kat2_streams(k, spdz)
    partner = [tuple(x) for x in k["partner_diffs"]]
    odo, own, products = O.compute_output_delivery_object(
        spdz, O.strip_macs(share_data), masks, triples, [partner], k["player_id"])
    assert [list(x) for x in own] == k["expected_own_diffs"]
    assert products == k["expected_products"]
    n_pairs = 2 * len(k["secret_values"])
    assert str(O.operation_id(uuid.UUID(k["request_id"]), n_pairs)) == k["expected_operation_id"]
    mv = k["input_mask_values"]
    expected = O.OutputDeliveryObject(
        b"".join(spdz.to_gfp(v) for v in k["secret_values"]),
        b"".join(spdz.to_gfp(v) for v in mv[0::2]),
        b"".join(spdz.to_gfp(v) for v in mv[1::2]),
        b"".join(spdz.to_gfp(v) for v in k["expected_products"][0::2]),
        b"".join(spdz.to_gfp(v) for v in k["expected_products"][1::2]))
    assert odo == expected


def _abs_next_long(rng):
    return abs(rng.getrandbits(64) - 2 ** 63)


def test_kat3_verify_pass_and_fail():
    util = O.ClientSecretShareUtil.of(P, R, RINV)
    rng = random.Random(42)
    n = 5
    s = [_abs_next_long(rng) for _ in range(n)]
    r = [_abs_next_long(rng) for _ in range(n)]
    v = [_abs_next_long(rng) for _ in range(n)]
    w = [a * b for a, b in zip(s, r)]
    u = [a * b for a, b in zip(v, r)]
    util.verify_secrets(s, r, u, v, w)
    w[-1] -= 10
    with pytest.raises(O.IntegrityVerificationException) as ei:
        util.verify_secrets(s, r, u, v, w)
    assert str(ei.value).startswith("Verification of secret has failed")


def test_odo_length_invariant():
    # OutputDeliveryObjectTest.java:19-90
    with pytest.raises(O.IllegalArgumentException, match="same length"):
        O.OutputDeliveryObject(bytes(16), bytes(16), bytes(32), bytes(16), bytes(16))


def _share2(spdz, rng, x, t1, t2):
    mask = rng.getrandbits(P.bit_count() - 1)
    t1.append(spdz.to_gfp(mask))
    t2.append(spdz.to_gfp((x - mask) % P))


def _odos_for(spdz, rng, secrets):
    """DefaultAmphoraClientTest.getOutputDeliveryObjectsForSecrets :782-820."""
    b = [[[] for _ in range(5)] for _ in range(2)]
    for s in secrets:
        r = rng.getrandbits(64) - 2 ** 63  # nextLong: may be negative
        v = rng.getrandbits(64) - 2 ** 63
        for k, x in enumerate((s, r, v, s * r % P, v * r % P)):
            _share2(spdz, rng, x, b[0][k], b[1][k])
    return [O.OutputDeliveryObject(*[b"".join(b[j][k]) for k in range(5)]) for j in range(2)]


def test_roundtrip_create_secret(spdz):
    """DefaultAmphoraClientTest.java:193-235: sum(masks) + masked == secret."""
    util = O.ClientSecretShareUtil.of(P, R, RINV)
    rng = random.Random(1)
    for _ in range(10):
        size = rng.randrange(1, 200)
        secrets = [rng.randrange(2 ** 63) for _ in range(size)]
        masks = [rng.getrandbits(P.bit_length()) % P for _ in range(size)]
        odos = _odos_for(spdz, rng, masks)
        masked = O.create_secret_masked_inputs(util, secrets, odos)
        for j in range(size):
            m = sum(spdz.from_gfp(o.secret_shares[16 * j:16 * j + 16]) for o in odos) % P
            assert (m + spdz.from_gfp(masked[j])) % P == secrets[j]


def test_roundtrip_get_secret(spdz):
    """DefaultAmphoraClientTest.java:254-271: recovered data == secrets."""
    util = O.ClientSecretShareUtil.of(P, R, RINV)
    rng = random.Random(2)
    for _ in range(10):
        size = rng.randrange(1, 200)
        secrets = [rng.randrange(2 ** 63) for _ in range(size)]
        assert O.verify_output_delivery_objects(util, _odos_for(spdz, rng, secrets)) == secrets


def test_recombine_empty_and_ragged(spdz):
    util = O.ClientSecretShareUtil.of(P, R, RINV)
    assert util.recombine_object([]) == []
    assert util.recombine_object([b"", b""]) == []
    # a trailing partial word is ignored (length / WORD_WIDTH)
    one = spdz.to_gfp(5) + b"\x01\x02"
    assert util.recombine_object([one, spdz.to_gfp(7) + b"\x00\x00"]) == [12]


# ---- the C restatement agrees with the Python restatement on the golden vectors


def _load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name), allow_pickle=False)


def _cases(golden_dir):
    with open(os.path.join(golden_dir, "manifest.json")) as f:
        return json.load(f)["cases"]


@pytest.mark.parametrize("idx", range(4))
def test_c_oracle_matches_golden(golden_dir, idx):
    case = _cases(golden_dir)[idx]
    d = _load(golden_dir, case["file"])
    n = case["parties"]
    F = coracle.test_field(threads=2)
    for tag in ("honest", "fault", "noncanon"):
        buf = d["rv_%s_odo" % tag]
        odos = [tuple(buf[k, j] for k in range(5)) for j in range(n)]
        y, ff = F.recombine_verify(odos)
        assert ff == d["rv_%s_first_fail" % tag][0]
        assert np.array_equal(y, d["rv_%s_secrets" % tag])
    mo = d["mask_odo"]
    out, ff = F.mask_input(d["mask_secrets"], [tuple(mo[k, j] for k in range(5)) for j in range(n)])
    assert ff == -1 and np.array_equal(out, d["mask_out"])
    mf = d["mask_fault_odo"]
    _, ff = F.mask_input(d["mask_secrets"], [tuple(mf[k, j] for k in range(5)) for j in range(n)])
    assert ff == d["mask_fault_first_fail"][0]
    key = int.from_bytes(d["conv_mac_key"].tobytes(), "little")
    for z in (0, 1):
        out = F.convert_share(d["conv_masked"], d["conv_tuples"], key, bool(z))
        assert np.array_equal(out, d["conv_out_zero%d" % z])
    y, r, v, mag, neg = F.odo_pre(d["odo_share_data"], 32, d["odo_masks"], d["odo_triples"])
    for got, key_ in ((y, "odo_y"), (r, "odo_r"), (v, "odo_v"), (mag, "odo_diff_mag"),
                      (neg, "odo_diff_neg")):
        assert np.array_equal(got, d[key_]), key_
    mags = [mag] + [d["odo_partner_mag"][j] for j in range(n - 1)]
    negs = [neg] + [d["odo_partner_neg"][j] for j in range(n - 1)]
    opened = F.recombine_diffs(mags, negs)
    assert np.array_equal(opened, d["odo_opened"])
    for pid in (0, 1):
        w, u = F.odo_post(d["odo_opened"], d["odo_triples"], pid == 0)
        assert np.array_equal(w, d["odo_w_p%d" % pid]) and np.array_equal(u, d["odo_u_p%d" % pid])


def test_golden_vectors_reproducible(golden_dir):
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "make_golden", os.path.join(os.path.dirname(golden_dir), "..", "tools", "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    case = _cases(golden_dir)[2]
    d = mg.make_case(case["parties"], case["words"], case["seed"])
    ref = _load(golden_dir, case["file"])
    for k, v in d.items():
        assert np.array_equal(v, ref[k]), k


def test_c_oracle_synth_is_honest_and_faults():
    F = coracle.test_field(threads=4)
    for n in (1, 2, 3):
        odos, _ = F.synth_odos(seed=5, n=n, W=1000, noncanon_permille=20)
        y, ff = F.recombine_verify(odos)
        assert ff == -1
        odos, _ = F.synth_odos(seed=5, n=n, W=1000, fault_index=333)
        _, ff = F.recombine_verify(odos)
        assert ff == 333


def test_c_oracle_vs_python_random():
    """Independent spot check of the C oracle's Knuth-division mulmod against
    Python ints on synthetic 3-party ODOs."""
    F = coracle.test_field(threads=2)
    spdz = O.MpSpdzIntegrationUtils(P, R, RINV)
    util = O.ClientSecretShareUtil(P, R, RINV)
    odos, buf = F.synth_odos(seed=9, n=3, W=300, noncanon_permille=100)
    y, ff = F.recombine_verify(odos)
    po = [O.OutputDeliveryObject(*[buf[k, j].tobytes() for k in range(5)]) for j in range(3)]
    assert O.verify_output_delivery_objects(util, po) == [
        int.from_bytes(y[i].tobytes(), "little") for i in range(300)]


def test_package_field_constants_match_oracle():
    """bench.py and the tools take the field from amphora_amd.spdz, never
    from oracle/: both restate the same reference configuration."""
    from amphora_amd import spdz
    assert (spdz.TEST_PRIME, spdz.TEST_R, spdz.TEST_RINV) == (O.TEST_PRIME, O.TEST_R, O.TEST_RINV)
