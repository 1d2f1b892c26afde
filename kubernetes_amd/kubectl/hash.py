"""Content hashes for `kubectl create configmap|secret --append-hash`
(`pkg/kubectl/util/hash/hash.go`): SHA-256 over a canonical JSON encoding of the object's kind,
name, (type) and data, keys sorted as Go's encoding/json writes them; the first ten hex digits,
with 0 1 3 a e swapped for g h k m t so the suffix never looks like a number or a word."""
from __future__ import annotations

import hashlib
import json

_SWAP = str.maketrans({"0": "g", "1": "h", "3": "k", "a": "m", "e": "t"})


def _go_json(obj) -> str:
    """encoding/json.Marshal: compact, sorted map keys, UTF-8 kept, <>& and U+2028/9 escaped."""
    s = json.dumps(obj, sort_keys=True, separators=(",", ":"), ensure_ascii=False)
    for ch, esc in (("<", "\\u003c"), (">", "\\u003e"), ("&", "\\u0026"), (" ", "\\u2028"),
                    (" ", "\\u2029")):
        s = s.replace(ch, esc)
    return s


def encode_config_map(cm) -> str:
    return _go_json({"kind": "ConfigMap", "name": (cm.get("metadata") or {}).get("name", ""),
                     "data": cm.get("data") or {}})


def encode_secret(sec) -> str:
    """Secret data is already base64 in the API object, as []byte encodes in Go."""
    return _go_json({"kind": "Secret", "type": sec.get("type", ""), "name": (sec.get("metadata") or {}).get("name", ""),
                     "data": sec.get("data") or {}})


def encode_hash(hexdigest: str) -> str:
    if len(hexdigest) < 10:
        raise ValueError("the hex string must contain at least 10 characters")
    return hexdigest[:10].translate(_SWAP)


def config_map_hash(cm) -> str:
    return encode_hash(hashlib.sha256(encode_config_map(cm).encode()).hexdigest())


def secret_hash(sec) -> str:
    return encode_hash(hashlib.sha256(encode_secret(sec).encode()).hexdigest())
