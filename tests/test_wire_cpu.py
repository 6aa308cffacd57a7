"""JSON framing helpers of amphora_amd.wire that need no GPU: the structural
walk that finds the OutputDeliveryObject members of a VerifiableSecretShare
(amphora-common/.../VerifiableSecretShare.java:30-87) without building a JSON
tree for the base64 values."""
import json

from amphora_amd import wire


def _doc(tags, pretty):
    obj = {"secretId": "80fbba1b-3da8-4b1e-8a2c-cebd65229fad", "tags": tags}
    obj.update({k: k[0] * 8 for k in wire.ODO_FIELDS})
    return json.dumps(obj, indent=2 if pretty else None)


def test_members_are_top_level_only():
    tags = [{"key": "rShares", "value": "secretShares", "valueType": "STRING"},
            {"key": 'x"uShares"', "value": "vShares\\", "valueType": "STRING"}]
    for pretty in (False, True):
        text = _doc(tags, pretty)
        m = wire._top_level_members(text)
        assert set(m) == {"secretId", "tags"} | set(wire.ODO_FIELDS)
        for k in wire.ODO_FIELDS:
            v, s, e = wire._extract(text, m, k)
            assert v == k[0] * 8 and text[s:e].startswith('"%s"' % k)


def test_missing_and_null_members():
    text = json.dumps({"secretId": "x", "tags": [{"key": "wShares", "value": "1"}], "rShares": None})
    m = wire._top_level_members(text)
    assert wire._extract(text, m, "wShares")[0] is None  # only a tag is named so
    assert wire._extract(text, m, "rShares")[0] is None
    assert wire._extract(text, m, "uShares") == (None, -1, -1)


def test_odo_field_texts_and_word_counts():
    import pytest
    from amphora_amd import entities as E
    text = _doc([{"key": "uShares", "value": "x", "valueType": "STRING"}], pretty=True)
    vals, spans = wire.odo_field_texts(text)
    assert vals == [k[0] * 8 for k in wire.ODO_FIELDS]
    assert all(text[s:e].startswith('"%s"' % k) for (s, e), k in zip(spans, wire.ODO_FIELDS))
    sid, tags = wire.vss_metadata(text, spans)
    assert str(sid) == "80fbba1b-3da8-4b1e-8a2c-cebd65229fad" and tags[0]["key"] == "uShares"
    # 16 W bytes <-> 4 ceil(16 W / 3) characters with 0 / 2 / 1 '='
    import base64
    for W in (0, 1, 2, 3, 100):
        t = base64.b64encode(bytes(16 * W)).decode()
        assert wire.words_of_b64(len(t), t[-2:]) == W
    with pytest.raises(ValueError, match="whole number"):
        wire.words_of_b64(8, "==")  # 4 bytes
    with pytest.raises(E.IllegalArgumentException, match="rShares is marked non-null"):
        wire.odo_field_texts('{"secretShares":"AAAA"}')


def test_masked_input_records_framing():
    import json
    import uuid
    import numpy as np
    rec = np.frombuffer(b"A" * 22 + b"==" + b"B" * 22 + b"==", np.uint8).reshape(2, 24)
    sid = uuid.UUID("3bcf8308-8f50-4d24-a37b-b0075bb5e779")
    text = wire.records_to_masked_input_json(sid, rec, [("k", "v")])
    obj = json.loads(text)
    assert obj == {"secretId": str(sid), "data": [{"value": "A" * 22 + "=="}, {"value": "B" * 22 + "=="}],
                   "tags": [{"key": "k", "value": "v", "valueType": "STRING"}]}
    got, rest = wire._compact_records(text)
    assert np.array_equal(got, rec) and json.loads(rest)["data"] == []
    # anything but the compact layout falls back to the JSON parser
    assert wire._compact_records(json.dumps(obj, indent=1)) is None
    assert wire._compact_records(text.replace('"tags"', '"data2"').replace('"data2"', '"data"')) is None
    empty = wire.records_to_masked_input_json(sid, np.zeros((0, 24), np.uint8), [])
    assert wire._compact_records(empty)[0].shape == (0, 24)


def test_masked_input_words_sequence():
    import numpy as np
    import pytest
    from amphora_amd import entities as E
    w = np.arange(48, dtype=np.uint8).reshape(3, 16)
    s = E.MaskedInputWords(w)
    assert len(s) == 3 and s[1] == E.MaskedInputData.of(bytes(range(16, 32)))
    assert [d.value for d in s] == [bytes(r) for r in w] and s[1:].words.shape == (2, 16)
    assert s == [E.MaskedInputData.of(bytes(r)) for r in w]
    with pytest.raises(E.IllegalArgumentException, match="has to be 16 bytes"):
        E.MaskedInputWords(np.zeros((2, 15), np.uint8))
