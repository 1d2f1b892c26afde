"""Encryption at rest for stored API objects: value transformers + EncryptionConfig loader.

Parity:
  * `PrefixTransformers` — `staging/src/k8s.io/apiserver/pkg/storage/value/transformer.go:95-152`:
    writes use the FIRST provider (its prefix is prepended); reads try every provider whose
    prefix matches, so keys can be rotated by adding a new first provider. A read through a
    non-first provider is reported `stale` (the object should be rewritten).
  * providers — `staging/src/k8s.io/apiserver/pkg/server/options/encryptionconfig/config.go:39-42`
    (prefixes `k8s:enc:<provider>:v1:<key name>:`; identity has no prefix):
      aescbc    16-byte IV || AES-CBC/PKCS#7           (`encrypt/aes/aes.go:93-150`)
      aesgcm    12-byte nonce || AES-GCM, AAD = key    (`encrypt/aes/aes.go:51-83`)
      secretbox 24-byte nonce || XSalsa20-Poly1305     (`encrypt/secretbox/secretbox.go:36-68`)
      kms       envelope scheme, see `storage/kms.py`  (`encrypt/envelope/envelope.go:57-150`)
The ciphers run in native code (libkamd_crypto.so: OpenSSL EVP plus a C++ XSalsa20).
"""
from __future__ import annotations

import base64

import yaml

from ..native import crypto


class TransformError(Exception):
    pass


class Identity:
    """No transformation; refuses encrypted data so a later provider can read it
    (`encrypt/identity/identity.go:37-45`, used to migrate away from encryption)."""

    def from_storage(self, data, ctx):
        if data[:8] == b"k8s:enc:":
            raise TransformError("identity transformer tried to read encrypted data")
        return data

    def to_storage(self, data, ctx):
        return data


class AESCBC:
    def __init__(self, key: bytes):
        self.key = key

    def from_storage(self, data, ctx):
        if len(data) < 16:
            raise TransformError("the stored data was shorter than the required size")
        return crypto.aes_cbc_decrypt(self.key, data[:16], data[16:])

    def to_storage(self, data, ctx):
        iv = crypto.random_bytes(16)
        return iv + crypto.aes_cbc_encrypt(self.key, iv, data)


class AESGCM:
    def __init__(self, key: bytes):
        self.key = key

    def from_storage(self, data, ctx):
        if len(data) < 12:
            raise TransformError("the stored data was shorter than the required size")
        return crypto.aes_gcm_open(self.key, data[:12], data[12:], ctx)

    def to_storage(self, data, ctx):
        nonce = crypto.random_bytes(12)
        return nonce + crypto.aes_gcm_seal(self.key, nonce, data, ctx)


class Secretbox:
    def __init__(self, key: bytes):
        if len(key) != 32:
            raise TransformError("secretbox key must be 32 bytes")
        self.key = key

    def from_storage(self, data, ctx):
        if len(data) < 24 + 16:
            raise TransformError("the stored data was shorter than the required size")
        return crypto.secretbox_open(self.key, data[:24], data[24:])

    def to_storage(self, data, ctx):
        nonce = crypto.random_bytes(24)
        return nonce + crypto.secretbox_seal(self.key, nonce, data)


class PrefixTransformers:
    def __init__(self, providers):
        """providers: [(prefix bytes, transformer)] — the first one is used for writes."""
        if not providers:
            raise TransformError("no providers")
        self.providers = providers

    def from_storage(self, data: bytes, ctx: bytes):
        """Returns (plaintext, stale)."""
        for i, (prefix, t) in enumerate(self.providers):
            if data.startswith(prefix):
                try:
                    out = t.from_storage(data[len(prefix):], ctx)
                except (crypto.CryptoError, TransformError) as e:
                    if prefix:
                        raise TransformError(str(e))
                    continue
                return out, i != 0
        raise TransformError("no matching prefix found")

    def to_storage(self, data: bytes, ctx: bytes) -> bytes:
        prefix, t = self.providers[0]
        return prefix + t.to_storage(data, ctx)


ENC_PREFIX = b"k8s:enc:"


def _decode_secret(s: str) -> bytes:
    try:
        return base64.b64decode(s, validate=True)
    except Exception as e:
        raise TransformError(f"could not obtain secret for named key: {e}")


def _provider(p: dict, kms_dial=None):
    if len(p) != 1:
        raise TransformError("provider must contain exactly one of identity/aescbc/aesgcm/secretbox/kms")
    (kind, cfg), = p.items()
    cfg = cfg or {}
    if kind == "identity":
        return [(b"", Identity())]
    if kind in ("aescbc", "aesgcm", "secretbox"):
        cls = {"aescbc": AESCBC, "aesgcm": AESGCM, "secretbox": Secretbox}[kind]
        entries = cfg.get("keys") or []
        if not entries:
            raise TransformError(f"{kind} provider has no keys")
        out = []
        for k in entries:
            raw = _decode_secret(k["secret"])
            if kind != "secretbox" and len(raw) not in (16, 24, 32):
                raise TransformError(f"invalid key size {len(raw)} for {kind} key {k['name']}")
            out.append((f"k8s:enc:{kind}:v1:{k['name']}:".encode(), cls(raw)))
        return out
    if kind == "kms":
        from .kms import Envelope, KMSClient
        name = cfg.get("name")
        if not name:
            raise TransformError("kms provider needs a name")
        svc = (kms_dial or KMSClient)(cfg.get("endpoint") or cfg.get("configfile") or "")
        return [(f"k8s:enc:kms:v1:{name}:".encode(), Envelope(svc, int(cfg.get("cachesize") or 1000)))]
    raise TransformError(f"unknown provider {kind!r}")


def load_encryption_config(path_or_dict, kms_dial=None) -> dict:
    """EncryptionConfig -> {resource plural: PrefixTransformers}."""
    cfg = path_or_dict
    if isinstance(cfg, str):
        with open(cfg) as f:
            cfg = yaml.safe_load(f)
    if (cfg or {}).get("kind") not in ("EncryptionConfig", "EncryptionConfiguration"):
        raise TransformError("invalid configuration kind %r provided" % (cfg or {}).get("kind"))
    out = {}
    for rc in cfg.get("resources") or []:
        providers = []
        for p in rc.get("providers") or []:
            providers += _provider(p, kms_dial)
        t = PrefixTransformers(providers)
        for r in rc.get("resources") or []:
            out[r.split(".", 1)[0]] = t
    return out
