"""Serialization: JSON wire form and the etcd storage envelope.

Storage format parity: values stored under `/registry/...` are
  * protobuf media type: `k8s\\x00` magic + `runtime.Unknown{TypeMeta, Raw}` envelope
    (`staging/src/k8s.io/apimachinery/pkg/runtime/serializer/protobuf/protobuf.go:42`,
    `staging/src/k8s.io/apimachinery/pkg/runtime/types.go:112-124`), Raw = the v1 protobuf
    encoding of the object (`kubernetes_amd.api.protobuf`);
  * JSON media type: the plain JSON object (reference `--storage-media-type=application/json`).
"""
from __future__ import annotations

import json

JSON = "application/json"
PROTOBUF = "application/vnd.kubernetes.protobuf"
YAML = "application/yaml"
MAGIC = b"k8s\x00"

_enc = json.JSONEncoder(separators=(",", ":"), ensure_ascii=False, check_circular=False)
_dec = json.JSONDecoder()


def dumps(obj) -> str:
    return _enc.encode(obj)


def dumpb(obj) -> bytes:
    return _enc.encode(obj).encode()


def loads(b):
    if isinstance(b, (bytes, bytearray, memoryview)):
        b = bytes(b).decode()
    return _dec.decode(b)


class StorageCodec:
    """Encodes objects for the KV store. `media_type` mirrors `--storage-media-type`."""

    def __init__(self, media_type: str = JSON):
        self.media_type = media_type
        if media_type == PROTOBUF:
            from . import protobuf as _pb
            self._pb = _pb

    def encode(self, obj) -> bytes:
        if self.media_type == PROTOBUF:
            return self._pb.encode_storage(obj)
        return dumpb(obj)

    def decode(self, data: bytes):
        if data[:4] == MAGIC:
            from . import protobuf as _pb
            return _pb.decode_storage(data)
        return loads(data)
