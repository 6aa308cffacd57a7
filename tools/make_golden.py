"""Generate the committed golden fixtures under tests/golden/.

Run from the repo root:  python tools/make_golden.py
Uses ONLY the pure-Python oracle (oracle/amphora_oracle.py); the reference
(Java) cannot run in this container (no JDK), so the fixtures are anchored by
the reference's own known-answer tests, which tests/test_oracle_kat.py checks
this oracle against first:

* kat.json -- the literal decimal inputs/outputs of
  amphora-service/.../calculation/SecretShareUtilTest.java:68-107 (KAT-1) and
  amphora-service/.../calculation/OutputDeliveryServiceTest.java:55-175 (KAT-2),
  transcribed as data.
* vectors_n{2,3}.npz -- seeded random cases produced by the oracle for every
  row of SURVEY.md 8(a): honest, fault-injected and non-canonical inputs.
"""
from __future__ import annotations

import json
import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import amphora_oracle as O  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
P, R, RINV = O.TEST_PRIME, O.TEST_R, O.TEST_RINV


def kat_json():
    kat1 = {
        "source": "amphora-service/src/test/java/io/carbynestack/amphora/service/calculation/"
                  "SecretShareUtilTest.java:68-107",
        "mac_key": "-33717010807885571165607137982809795379",
        "masked_inputs": ["37371993412255263319479925008425883363", "0"],
        "input_masks": [["-82730997414791468496799367418496881908",
                         "-60557275363670854182192939229091375859"],
                        ["45359004002536205186084333850157344582",
                         "-48604663536222227589564560476962533035"]],
        "use_zero_input_as_data": False,
        "expected_share_words": ["-45359004002536205177319442410070998545",
                                 "-170814686092998134911558977038957876158",
                                 "45359004002536205186084333850157344582",
                                 "-48604663536222227589564560476962533035"],
        "note": "every value is taken mod p before toGfp, as in the test",
    }
    kat2 = {
        "source": "amphora-service/src/test/java/io/carbynestack/amphora/service/calculation/"
                  "OutputDeliveryServiceTest.java:55-175,285-382",
        "player_id": 0,
        "secret_values": [90, 142],
        "input_mask_values": [87, 111, 412, 313],
        "triples": [[80, 62, 3719], [72, 63, 32521], [141, 264, 56212], [19, 35, 612]],
        "expected_own_diffs": [[10, 25], [39, 24], [1, 148], [294, 377]],
        "partner_diffs": [[4, 63], [175, 136], [5, 106], [2, 27]],
        "expected_products": [12859, 91763, 95134, 138232],
        "request_id": "70297fd4-d412-4dbb-af05-6818fe0e687a",
        "expected_operation_id": "8065e700-9f48-36ba-ae8c-f881b28a28ef",
    }
    field = {"prime": str(P), "r": str(R), "r_inv": str(RINV),
             "source": "amphora-java-client/.../SecretShareUtilTest.java:24-28"}
    anchors = {"toGfp(1)": O.MpSpdzIntegrationUtils(P, R, RINV).to_gfp(1).hex(),
               "toGfp(90)": O.MpSpdzIntegrationUtils(P, R, RINV).to_gfp(90).hex(),
               "encoding": O.ENCODING}
    return {"field": field, "kat1": kat1, "kat2": kat2, "encoding_anchors": anchors}


def le(x):
    return int(x).to_bytes(16, "little")


def arr(words_bytes):
    b = b"".join(words_bytes)
    return np.frombuffer(b, np.uint8).reshape(-1, 16).copy() if b else np.zeros((0, 16), np.uint8)


def share_odos(spdz, rng, values_5, n, fault=None, noncanon=0.0):
    """values_5: list of 5 lists (y, r, v, w, u) of ints.  Additive N-party
    sharing (n-1 uniform, last = x - sum), toGfp-encoded -> (5, n, W, 16)."""
    W = len(values_5[0])
    out = np.zeros((5, n, W, 16), np.uint8)
    for k in range(5):
        for i in range(W):
            rest = values_5[k][i] % P
            for j in range(n):
                if j < n - 1:
                    sh = rng.randrange(P)
                    rest = (rest - sh) % P
                else:
                    sh = rest
                if fault is not None and k == 3 and i == fault and j == (1 if n > 1 else 0):
                    sh = (sh + 1) % P
                raw = (sh * R) % P
                if noncanon and rng.random() < noncanon and raw + P < 2 ** 128:
                    raw += P  # non-canonical word (>= p), as random-byte fixtures produce
                out[k, j, i] = np.frombuffer(raw.to_bytes(16, "little"), np.uint8)
    return out


def honest_values(rng, W, ys=None):
    ys = ys if ys is not None else [rng.randrange(P) for _ in range(W)]
    rs = [rng.randrange(P) for _ in range(W)]
    vs = [rng.randrange(P) for _ in range(W)]
    return [ys, rs, vs, [y * r % P for y, r in zip(ys, rs)], [v * r % P for v, r in zip(vs, rs)]]


def odos_from(buf):
    n = buf.shape[1]
    return [O.OutputDeliveryObject(*[buf[k, j].tobytes() for k in range(5)]) for j in range(n)]


def make_case(n, W, seed):
    rng = random.Random(seed)
    spdz = O.MpSpdzIntegrationUtils(P, R, RINV)
    util = O.ClientSecretShareUtil(P, R, RINV)
    d = {}
    # --- K_RV: download ODOs (honest, faulted at W//3, non-canonical words)
    secrets = [rng.randrange(P) if i % 2 else rng.randrange(2 ** 63) for i in range(W)]
    vals = honest_values(rng, W, secrets)
    for tag, fault, nc in (("honest", None, 0.0), ("fault", W // 3, 0.0), ("noncanon", None, 0.05)):
        buf = share_odos(spdz, rng, vals, n, fault, nc)
        d["rv_%s_odo" % tag] = buf
        try:
            ys = O.verify_output_delivery_objects(util, odos_from(buf))
            ff = -1
        except O.IntegrityVerificationException:
            ff = O.first_failing_index(P, *recombined_five(util, odos_from(buf)))
            ys = recombined_five(util, odos_from(buf))[0]
        d["rv_%s_secrets" % tag] = arr(le(y) for y in ys)
        d["rv_%s_first_fail" % tag] = np.array([ff], np.int64)
    # --- K_MASK: Input Mask ODOs + secrets -> masked inputs
    mvals = honest_values(rng, W)
    mask_buf = share_odos(spdz, rng, mvals, n)
    d["mask_odo"] = mask_buf
    d["mask_secrets"] = arr(le(s) for s in secrets)
    d["mask_out"] = arr(O.create_secret_masked_inputs(util, secrets, odos_from(mask_buf)))
    mask_fault = share_odos(spdz, rng, mvals, n, fault=W - 1)
    d["mask_fault_odo"] = mask_fault
    d["mask_fault_first_fail"] = np.array([W - 1 if W else -1], np.int64)
    # --- K_CONV: masked inputs + input mask tuples + mac key
    tuples = b"".join(le(rng.randrange(P) * R % P) + le(rng.randrange(P) * R % P) for _ in range(W))
    mac_key = rng.randrange(P)
    d["conv_masked"] = d["mask_out"]
    d["conv_tuples"] = np.frombuffer(tuples, np.uint8).reshape(-1, 32).copy() if W else np.zeros((0, 32), np.uint8)
    d["conv_mac_key"] = np.frombuffer(le(mac_key), np.uint8).copy()
    masks = [(tuples[32 * i:32 * i + 16], tuples[32 * i + 16:32 * i + 32]) for i in range(W)]
    for flag in (False, True):
        sd = O.convert_to_secret_share(spdz, [x.tobytes() for x in d["mask_out"]], str(mac_key), masks, flag)
        d["conv_out_zero%d" % int(flag)] = np.frombuffer(sd, np.uint8).reshape(-1, 32).copy() if W else np.zeros((0, 32), np.uint8)
    # --- K_ODO_PRE / POST: share data (32 B/word), 2W masks, 2W triples
    share_data = d["conv_out_zero0"]
    mstream = b"".join(le(rng.randrange(P) * R % P) + le(rng.randrange(P) * R % P) for _ in range(2 * W))
    tstream = b"".join(le(rng.randrange(P) * R % P) for _ in range(2 * W * 6))
    d["odo_share_data"] = share_data
    d["odo_masks"] = np.frombuffer(mstream, np.uint8).reshape(-1, 32).copy() if W else np.zeros((0, 32), np.uint8)
    d["odo_triples"] = np.frombuffer(tstream, np.uint8).reshape(-1, 96).copy() if W else np.zeros((0, 96), np.uint8)
    masks = O.parse_input_masks(mstream)
    triples = O.parse_triples(tstream)
    y_raw, r_raw, v_raw, pairs = O.odo_factor_pairs(spdz, O.strip_macs(share_data.tobytes()), masks)
    own = O.beaver_diffs(spdz, pairs, triples)
    d["odo_y"], d["odo_r"], d["odo_v"] = arr([y_raw]), arr([r_raw]), arr([v_raw])
    mag = np.zeros((2 * W, 2, 16), np.uint8)
    neg = np.zeros((2 * W, 2), np.uint8)
    for k, (a, b) in enumerate(own):
        for c, x in enumerate((a, b)):
            mag[k, c] = np.frombuffer(le(abs(x)), np.uint8)
            neg[k, c] = 1 if x < 0 else 0
    d["odo_diff_mag"], d["odo_diff_neg"] = mag, neg
    partners = [[(rng.randrange(-P + 1, P), rng.randrange(-P + 1, P)) for _ in range(2 * W)]
                for _ in range(n - 1)]
    opened = O.recombine_diffs(P, [own] + partners)
    op = np.zeros((2 * W, 2, 16), np.uint8)
    for k, (a, b) in enumerate(opened):
        op[k, 0] = np.frombuffer(le(a % P), np.uint8)
        op[k, 1] = np.frombuffer(le(b % P), np.uint8)
    d["odo_opened"] = op
    pmag = np.zeros((n - 1, 2 * W, 2, 16), np.uint8)
    pneg = np.zeros((n - 1, 2 * W, 2), np.uint8)
    for j, lst in enumerate(partners):
        for k, (a, b) in enumerate(lst):
            for c, x in enumerate((a, b)):
                pmag[j, k, c] = np.frombuffer(le(abs(x)), np.uint8)
                pneg[j, k, c] = 1 if x < 0 else 0
    d["odo_partner_mag"], d["odo_partner_neg"] = pmag, pneg
    for pid in (0, 1):
        prods = [O.multiply_shared_secrets(spdz, triples[k], opened[k][0], opened[k][1], pid)
                 for k in range(2 * W)]
        d["odo_w_p%d" % pid] = arr(spdz.to_gfp(prods[2 * i]) for i in range(W))
        d["odo_u_p%d" % pid] = arr(spdz.to_gfp(prods[2 * i + 1]) for i in range(W))
    return d


def recombined_five(util, odos):
    return (util.recombine_object([o.secret_shares for o in odos]),
            util.recombine_object([o.r_shares for o in odos]),
            util.recombine_object([o.u_shares for o in odos]),
            util.recombine_object([o.v_shares for o in odos]),
            util.recombine_object([o.w_shares for o in odos]))


def main():
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, "kat.json"), "w") as f:
        json.dump(kat_json(), f, indent=1)
    manifest = {"generator": "tools/make_golden.py", "oracle": "oracle/amphora_oracle.py",
                "encoding": O.ENCODING, "field": {"prime": str(P), "r": str(R), "r_inv": str(RINV)},
                "cases": []}
    for n, W, seed in ((2, 1, 7), (2, 257, 42), (3, 130, 43), (4, 33, 44)):
        d = make_case(n, W, seed)
        name = "vectors_n%d_w%d.npz" % (n, W)
        np.savez_compressed(os.path.join(OUT, name), **d)
        manifest["cases"].append({"file": name, "parties": n, "words": W, "seed": seed,
                                  "keys": sorted(d.keys())})
    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
