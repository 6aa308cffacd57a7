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
