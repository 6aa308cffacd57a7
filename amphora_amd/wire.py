"""Wire formats of the hot path's inputs and outputs, with the byte arrays
base64-coded on the GPU (amph_base64_*).

* VerifiableSecretShare JSON (GET /secret-shares/{id}):
  amphora-common/.../VerifiableSecretShare.java:30-87 -- the Metadata fields
  (secretId, tags) followed by the OutputDeliveryObject fields (secretShares,
  rShares, vShares, wShares, uShares) as base64 strings; pretty form pinned by
  VerifiableSecretTest.java:41-90 (Jackson's DefaultPrettyPrinter).
* OutputDeliveryObject JSON (GET /input-masks): the five base64 fields.
* MaskedInput JSON (POST /masked-inputs): MaskedInput.java:25-62 --
  {"secretId", "data": [{"value": base64(16 bytes)}, ...], "tags"}; each word
  is coded on its own (24 chars), the records are framed with numpy.

Large payloads: the base64 spans are located by a structural walk of the
outermost object that skips strings whole (no JSON tree is built for them);
only the small remainder goes through json.loads.
"""
from __future__ import annotations

import json
import re
import uuid
from typing import List, Tuple

import numpy as np

from . import _lib
from .entities import (IllegalArgumentException, MaskedInput, MaskedInputData, MaskedInputWords,
                       OutputDeliveryObject)

ODO_FIELDS = ("secretShares", "rShares", "vShares", "wShares", "uShares")


def _tag_obj(t):
    if isinstance(t, dict):
        d = dict(t)
    else:
        k, v = t[0], t[1]
        d = {"key": k, "value": v, "valueType": t[2] if len(t) > 2 else "STRING"}
    d.setdefault("valueType", "STRING")
    return {"key": d["key"], "value": d["value"], "valueType": d["valueType"]}


def _pretty_tags(tags, indent="  "):
    if not tags:
        return "[ ]"
    items = []
    for t in tags:
        o = _tag_obj(t)
        items.append("{\n" + ",\n".join('%s  "%s" : %s' % (indent, k, json.dumps(o[k])) for k in o)
                     + "\n" + indent + "}")
    return "[ " + ", ".join(items) + " ]"


def vss_to_json(ctx: _lib.Context, secret_id: uuid.UUID, tags, odo: OutputDeliveryObject,
                pretty: bool = True) -> str:
    """VerifiableSecretShare -> JSON (Jackson's pretty printer layout when pretty)."""
    b64 = [ctx.base64_encode(bytes(f)).decode("ascii") for f in odo.fields()]
    if pretty:
        lines = ['  "secretId" : "%s"' % secret_id, '  "tags" : %s' % _pretty_tags(tags)]
        lines += ['  "%s" : "%s"' % (k, v) for k, v in zip(ODO_FIELDS, b64)]
        return "{\n" + ",\n".join(lines) + "\n}"
    head = {"secretId": str(secret_id), "tags": [_tag_obj(t) for t in tags]}
    body = ",".join('"%s":"%s"' % (k, v) for k, v in zip(ODO_FIELDS, b64))
    return json.dumps(head, separators=(",", ":"))[:-1] + "," + body + "}"


def odo_to_json(ctx: _lib.Context, odo: OutputDeliveryObject) -> str:
    b64 = [ctx.base64_encode(bytes(f)).decode("ascii") for f in odo.fields()]
    return "{" + ",".join('"%s":"%s"' % (k, v) for k, v in zip(ODO_FIELDS, b64)) + "}"


_SIGNIFICANT = re.compile(r'["{}\[\]]')


def _string_end(text: str, j: int) -> int:
    """Index of the quote closing the JSON string that opens at text[j]."""
    k = j + 1
    while True:
        k = text.find('"', k)
        if k < 0:
            raise ValueError("malformed JSON: unterminated string")
        b = k - 1
        while text[b] == "\\":
            b -= 1
        if (k - 1 - b) % 2 == 0:  # an even run of backslashes: the quote is not escaped
            return k
        k += 1


def _top_level_members(text: str):
    """{key: (key_start, value_start)} of the outermost object's members.

    Only the structure is walked: strings are skipped whole with str.find (the
    base64 values hold no quotes), so a 100 MB member costs a few calls, and a
    key nested deeper -- e.g. a tag whose key or value is "rShares" -- is not
    taken for a member of the object itself."""
    members, depth, pos = {}, 0, 0
    while True:
        m = _SIGNIFICANT.search(text, pos)
        if m is None:
            break
        c, i = m.group(), m.start()
        if c == '"':
            e = _string_end(text, i)
            if depth == 1:
                j = e + 1
                while j < len(text) and text[j] in " \t\r\n":
                    j += 1
                if j < len(text) and text[j] == ":":
                    members.setdefault(text[i + 1:e], (i, j + 1))
            pos = e + 1
        elif c in "{[":
            depth += 1
            pos = i + 1
        else:
            depth -= 1
            pos = i + 1
            if depth == 0:
                break
    return members


def _extract(text: str, members, key: str) -> Tuple[str, int, int]:
    """The string value of top-level member `key`: (value, member start, end)."""
    if key not in members:
        return None, -1, -1
    i, j = members[key]
    while j < len(text) and text[j] in " \t\r\n":
        j += 1
    if text.startswith("null", j):
        return None, i, j + 4
    if j >= len(text) or text[j] != '"':
        raise ValueError("field %s is not a string" % key)
    k = _string_end(text, j)
    return text[j + 1:k], i, k + 1


def _odo_from_text(ctx: _lib.Context, text: str):
    vals, spans = [], []
    members = _top_level_members(text)
    for k in ODO_FIELDS:
        v, s, e = _extract(text, members, k)
        if v is None:
            # Lombok @NonNull through Jackson's ValueInstantiationException
            raise IllegalArgumentException("%s is marked non-null but is null" % k)
        vals.append(ctx.base64_decode(v))
        spans.append((s, e))
    return OutputDeliveryObject(*vals), spans


def odo_from_json(ctx: _lib.Context, text: str) -> OutputDeliveryObject:
    return _odo_from_text(ctx, text)[0]


def vss_from_json(ctx: _lib.Context, text: str):
    """JSON -> (secret_id, tags, OutputDeliveryObject); unknown fields ignored
    (VSSDeserializer: FAIL_ON_UNKNOWN_PROPERTIES disabled)."""
    odo, spans = _odo_from_text(ctx, text)
    sid, tags = vss_metadata(text, spans)
    return sid, tags, odo


def vss_metadata(text: str, spans):
    """(secretId, tags) of a VerifiableSecretShare body with the ODO member
    spans cut out (json.loads on the small remainder only)."""
    rest, pos = [], 0
    for s, e in sorted(spans):
        rest.append(text[pos:s])
        pos = e
        # drop the separating comma that followed the removed member, if any
        while pos < len(text) and text[pos] in " \t\r\n":
            pos += 1
        if pos < len(text) and text[pos] == ",":
            pos += 1
    rest.append(text[pos:])
    small = re.sub(r",\s*}\s*$", "}", "".join(rest).strip())
    meta = json.loads(small) if small else {}
    if meta.get("secretId") is None:
        raise IllegalArgumentException("secretId is marked non-null but is null")
    return uuid.UUID(meta["secretId"]), list(meta.get("tags") or [])


def odo_field_texts(text: str):
    """The five base64 member strings of a VerifiableSecretShare /
    OutputDeliveryObject JSON body, in ODO order, without decoding them (for
    the fused K_RV / K_MASK wire kernels); also returns the spans removed."""
    members = _top_level_members(text)
    vals, spans = [], []
    for k in ODO_FIELDS:
        v, s, e = _extract(text, members, k)
        if v is None:
            raise IllegalArgumentException("%s is marked non-null but is null" % k)
        vals.append(v)
        spans.append((s, e))
    return vals, spans


def words_of_b64(nchars: int, last2: str) -> int:
    """16-byte words held by a base64 field of nchars characters ending in
    last2 (its padding); ValueError unless it is a whole number of words."""
    if nchars % 4:
        raise ValueError("base64 input length must be a multiple of 4")
    nbytes = 3 * nchars // 4 - (last2[-2:].count("=") if nchars else 0)
    if nbytes % 16:
        raise ValueError("base64 field of %d bytes is not a whole number of 16-byte words" % nbytes)
    return nbytes // 16


def records_to_masked_input_json(secret_id, records, tags) -> str:
    """MaskedInput JSON from the (W, 24) base64 records of the masked words
    (what amph_mask_input_b64 writes), framed as masked_input_to_json does."""
    rec = np.ascontiguousarray(records, np.uint8).reshape(-1, 24)
    W = rec.shape[0]
    if W:
        frame = np.empty((W, 37), np.uint8)
        frame[:, :10] = np.frombuffer(b'{"value":"', np.uint8)
        frame[:, 10:34] = rec
        frame[:, 34:37] = np.frombuffer(b'"},', np.uint8)
        data = b"[" + frame.tobytes()[:-1] + b"]"
    else:
        data = b"[]"
    tj = json.dumps([_tag_obj(t) for t in tags], separators=(",", ":"))
    return '{"secretId":"%s","data":%s,"tags":%s}' % (secret_id, data.decode("ascii"), tj)


def masked_input_to_json(ctx: _lib.Context, mi: MaskedInput) -> str:
    """MaskedInput -> compact JSON; the per-word base64 runs on the GPU and
    the {"value":"..."} records are framed with numpy (37 B per word)."""
    W = len(mi.data)
    if W:
        words = mi.data.words if hasattr(mi.data, "words") else \
            np.frombuffer(b"".join(d.value for d in mi.data), np.uint8).reshape(W, 16)
        rec = ctx.base64_encode_words(words)
        frame = np.empty((W, 37), np.uint8)
        frame[:, :10] = np.frombuffer(b'{"value":"', np.uint8)
        frame[:, 10:34] = rec
        frame[:, 34:37] = np.frombuffer(b'"},', np.uint8)
        data = b"[" + frame.tobytes()[:-1] + b"]"
    else:
        data = b"[]"
    tags = json.dumps([_tag_obj(t) for t in mi.tags], separators=(",", ":"))
    return '{"secretId":"%s","data":%s,"tags":%s}' % (mi.secret_id, data.decode("ascii"), tags)


_RECORD = np.frombuffer(b'{"value":"', np.uint8)


def _compact_records(text: str):
    """The (W, 24) base64 records of a MaskedInput body in the compact layout
    (what masked_input_to_json and Jackson's default writer produce:
    "data":[{"value":"<24>"},...]) located without a JSON tree, plus the text
    with the data array emptied; None for any other layout."""
    k = text.find('"data":[')
    if k < 0 or text.count('"data"') != 1:
        return None
    lb = k + len('"data":')
    rb = text.find("]", lb)
    if rb < 0:
        return None
    span = text[lb + 1:rb]
    if not span:
        return np.zeros((0, 24), np.uint8), text[:lb] + "[]" + text[rb + 1:]
    if (len(span) + 1) % 37:
        return None
    b = np.frombuffer((span + ",").encode("ascii", errors="replace"), np.uint8).reshape(-1, 37)
    if not (np.array_equal(b[:, :10], np.broadcast_to(_RECORD, (b.shape[0], 10)))
            and (b[:, 34] == ord('"')).all() and (b[:, 35] == ord("}")).all() and (b[:, 36] == ord(",")).all()):
        return None
    return np.ascontiguousarray(b[:, 10:34]), text[:lb] + "[]" + text[rb + 1:]


def masked_input_from_json(ctx: _lib.Context, text: str) -> MaskedInput:
    fast = _compact_records(text)
    if fast is not None:  # the records go to the GPU decoder as one array
        rec, rest = fast
        obj = json.loads(rest)
        if obj.get("secretId") is None:
            raise IllegalArgumentException("secretId is marked non-null but is null")
        words = ctx.base64_decode_words(rec) if rec.shape[0] else np.zeros((0, 16), np.uint8)
        return MaskedInput(uuid.UUID(obj["secretId"]), MaskedInputWords(words), list(obj.get("tags") or []))
    obj = json.loads(text)
    if obj.get("secretId") is None:
        raise IllegalArgumentException("secretId is marked non-null but is null")
    values = [d["value"] for d in (obj.get("data") or [])]
    if values and all(isinstance(v, str) and len(v) == 24 for v in values):
        rec = np.frombuffer("".join(values).encode("ascii"), np.uint8).reshape(-1, 24)
        words = ctx.base64_decode_words(rec)
        data = [MaskedInputData.of(bytes(w)) for w in words]
    else:  # MaskedInputData.of enforces the 16-byte length with the reference message
        data = [MaskedInputData.of(ctx.base64_decode(v)) for v in values]
    return MaskedInput(uuid.UUID(obj["secretId"]), data, list(obj.get("tags") or []))


# ---- MultiplicationExchangeObject (POST /inter-vcp/open) ------------------------
# amphora-common/.../MultiplicationExchangeObject.java:20-39: {operationId,
# playerId, interimValues: [FactorPair{a, b}]}, the BigIntegers as JSON numbers
# (Jackson defaults, field declaration order).  The interimValues array is
# coded on the GPU (amph_exchange_*); the two scalar fields around it here.
def exchange_to_json(ctx: _lib.Context, operation_id: uuid.UUID, player_id: int, mag, neg) -> bytes:
    """Own signed diffs (amph_odo_pre layout) -> compact JSON, byte-identical to
    Jackson's default serialisation of the MultiplicationExchangeObject."""
    arr = ctx.exchange_encode(mag, neg)
    if not isinstance(arr, bytes):  # device tensors -> host bytes
        out, n = arr
        arr = out[: int(n.item())].cpu().numpy().tobytes()
    return exchange_body(operation_id, player_id, arr)


def exchange_body(operation_id: uuid.UUID, player_id: int, interim_values: bytes) -> bytes:
    """The MultiplicationExchangeObject JSON around an interimValues array text
    (as amph_exchange_encode / amph_party_text write it)."""
    head = '{"operationId":"%s","playerId":%d,"interimValues":' % (operation_id, int(player_id))
    return head.encode() + bytes(interim_values) + b"}"


def exchange_span(text) -> Tuple[uuid.UUID, int, int, int]:
    """(operationId, playerId, lb, rb): text[lb:rb + 1] is the interimValues array."""
    text = text.encode() if isinstance(text, str) else bytes(text)
    return _exchange_split(text)


def _exchange_split(text: bytes):
    k = text.find(b'"interimValues"')
    lb = text.find(b"[", k) if k >= 0 else -1
    rb = text.rfind(b"]")
    if k < 0 or lb < 0 or rb < lb:
        raise IllegalArgumentException("interimValues is marked non-null but is null")
    meta = json.loads(text[:lb] + b"[]" + text[rb + 1:])
    for f in ("operationId", "playerId"):
        if meta.get(f) is None:
            raise IllegalArgumentException("%s is marked non-null but is null" % f)
    return uuid.UUID(meta["operationId"]), int(meta["playerId"]), lb, rb


def exchange_header(text) -> Tuple[uuid.UUID, int]:
    """(operationId, playerId) of a MultiplicationExchangeObject JSON."""
    text = text.encode() if isinstance(text, str) else bytes(text)
    op, pid, _, _ = _exchange_split(text)
    return op, pid


def exchange_from_json(ctx: _lib.Context, text, npairs: int):
    """JSON -> (operationId, playerId, mag (P,2,16), neg (P,2)); the array is
    parsed on the GPU (ValueError on a malformed number or pair count)."""
    text = text.encode() if isinstance(text, str) else bytes(text)
    op, pid, lb, rb = _exchange_split(text)
    mag, neg = ctx.exchange_decode(text[lb:rb + 1], npairs)
    return op, pid, mag, neg
