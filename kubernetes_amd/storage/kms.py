"""KMS envelope provider for encryption at rest.

Parity: `staging/src/k8s.io/apiserver/pkg/storage/value/encrypt/envelope/envelope.go:57-150` —
each write gets a fresh 32-byte data key (DEK); the DEK is wrapped by the key-management
service and stored in front of the payload as `u16be len || wrapped DEK || aescbc(DEK, data)`;
an LRU maps wrapped DEKs to ready transformers so reads rarely call the service.

The service is reached over gRPC on a unix socket with the KeyManagementService shape
(Version / Encrypt / Decrypt). `LocalKMS` is a small in-process implementation of that
service (AES-256-GCM wrapping key) for local-up clusters and tests.
"""
from __future__ import annotations

import os
from collections import OrderedDict

from ..native import crypto
from .value import AESCBC, TransformError


class Envelope:
    def __init__(self, service, cache_size=1000):
        self.service = service
        self.cache: OrderedDict = OrderedDict()
        self.cache_size = cache_size or 1000

    def _remember(self, wrapped, t):
        self.cache[wrapped] = t
        if len(self.cache) > self.cache_size:
            self.cache.popitem(last=False)

    def _transformer(self, wrapped: bytes):
        t = self.cache.get(wrapped)
        if t is not None:
            self.cache.move_to_end(wrapped)
            return t
        t = AESCBC(self.service.decrypt(wrapped))
        self._remember(wrapped, t)
        return t

    def from_storage(self, data, ctx):
        if len(data) < 2:
            raise TransformError("invalid data encountered by envelope transformer")
        n = int.from_bytes(data[:2], "big")
        if n + 2 > len(data):
            raise TransformError("invalid data encountered by envelope transformer, length longer than available bytes")
        return self._transformer(bytes(data[2:2 + n])).from_storage(data[2 + n:], ctx)

    def to_storage(self, data, ctx):
        dek = crypto.random_bytes(32)
        wrapped = self.service.encrypt(dek)
        t = AESCBC(dek)
        self._remember(wrapped, t)
        return len(wrapped).to_bytes(2, "big") + wrapped + t.to_storage(data, ctx)


_API = None
SERVICE = "v1beta1.KeyManagementService"


def api():
    global _API
    if _API is None:
        from ..utils.protodesc import build
        _API = build("v1beta1", "kms/v1beta1/service.proto", {
            "VersionRequest": [("version", 1, "string", "opt", None)],
            "VersionResponse": [("version", 1, "string", "opt", None), ("runtime_name", 2, "string", "opt", None),
                                ("runtime_version", 3, "string", "opt", None)],
            "DecryptRequest": [("version", 1, "string", "opt", None), ("cipher", 2, "bytes", "opt", None)],
            "DecryptResponse": [("plain", 1, "bytes", "opt", None)],
            "EncryptRequest": [("version", 1, "string", "opt", None), ("plain", 2, "bytes", "opt", None)],
            "EncryptResponse": [("cipher", 1, "bytes", "opt", None)],
        })
    return _API


class KMSClient:
    """Blocking client: envelope calls sit on the (synchronous) storage encode path."""

    def __init__(self, endpoint: str, timeout=3.0):
        import grpc
        if not endpoint:
            raise TransformError("kms provider needs an endpoint (unix:///path)")
        target = endpoint if endpoint.startswith("unix:") else "unix://" + endpoint
        self.channel = grpc.insecure_channel(target)
        self.timeout = timeout
        a = self.api = api()

        def method(name, req, resp):
            return self.channel.unary_unary(f"/{SERVICE}/{name}", request_serializer=req.SerializeToString,
                                            response_deserializer=resp.FromString)
        self._enc = method("Encrypt", a["EncryptRequest"], a["EncryptResponse"])
        self._dec = method("Decrypt", a["DecryptRequest"], a["DecryptResponse"])
        self._ver = method("Version", a["VersionRequest"], a["VersionResponse"])

    def version(self):
        r = self._ver(self.api["VersionRequest"](version="v1beta1"), timeout=self.timeout)
        return r.version, r.runtime_name

    def encrypt(self, plain: bytes) -> bytes:
        return self._enc(self.api["EncryptRequest"](version="v1beta1", plain=plain), timeout=self.timeout).cipher

    def decrypt(self, cipher: bytes) -> bytes:
        return self._dec(self.api["DecryptRequest"](version="v1beta1", cipher=cipher), timeout=self.timeout).plain


class LocalKMS:
    """In-process KeyManagementService on a unix socket (wrapping key = AES-256-GCM)."""

    def __init__(self, socket_path: str, wrapping_key: bytes | None = None):
        self.path = socket_path
        self.wrapping_key = wrapping_key or crypto.random_bytes(32)
        self.server = None
        self.calls = {"Encrypt": 0, "Decrypt": 0}

    def start(self):
        import grpc
        from concurrent import futures
        a = api()
        if os.path.exists(self.path):
            os.unlink(self.path)

        def enc(req, ctx):
            self.calls["Encrypt"] += 1
            n = crypto.random_bytes(12)
            return a["EncryptResponse"](cipher=n + crypto.aes_gcm_seal(self.wrapping_key, n, req.plain))

        def dec(req, ctx):
            self.calls["Decrypt"] += 1
            c = req.cipher
            return a["DecryptResponse"](plain=crypto.aes_gcm_open(self.wrapping_key, c[:12], c[12:]))

        def ver(req, ctx):
            return a["VersionResponse"](version="v1beta1", runtime_name="kamd-local-kms", runtime_version="0.1")

        def h(fn, req, resp):
            return grpc.unary_unary_rpc_method_handler(fn, request_deserializer=req.FromString,
                                                       response_serializer=resp.SerializeToString)
        handler = grpc.method_handlers_generic_handler(SERVICE, {
            "Encrypt": h(enc, a["EncryptRequest"], a["EncryptResponse"]),
            "Decrypt": h(dec, a["DecryptRequest"], a["DecryptResponse"]),
            "Version": h(ver, a["VersionRequest"], a["VersionResponse"]),
        })
        self.server = grpc.server(futures.ThreadPoolExecutor(max_workers=2))
        self.server.add_generic_rpc_handlers((handler,))
        self.server.add_insecure_port("unix://" + self.path)
        self.server.start()
        return self

    def stop(self):
        if self.server is not None:
            self.server.stop(0)
