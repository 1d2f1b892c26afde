"""Encryption at rest (storage value transformers) and the native crypto library.

Parity: `staging/src/k8s.io/apiserver/pkg/storage/value/transformer_test.go`,
`encrypt/aes/aes_test.go`, `encrypt/secretbox/secretbox_test.go`, `encrypt/envelope/envelope_test.go`.
"""
import base64
import os

import pytest

from kubernetes_amd.apiserver.server import APIServer
from kubernetes_amd.client.rest import Client
from kubernetes_amd.native import crypto
from kubernetes_amd.storage import value as v
from kubernetes_amd.storage.kms import KMSClient, LocalKMS
from kubernetes_amd.storage.remote import StoreServer


def b64(n, seed=1):
    return base64.b64encode(bytes((seed * 7 + i) % 256 for i in range(n))).decode()


def config(*providers, resources=("secrets",)):
    return {"kind": "EncryptionConfig", "apiVersion": "v1",
            "resources": [{"resources": list(resources), "providers": list(providers)}]}


SECRET = {"apiVersion": "v1", "kind": "Secret", "metadata": {"name": "s1", "namespace": "default"},
          "data": {"password": base64.b64encode(b"hunter2-plaintext-marker").decode()}}


def test_secretbox_matches_nacl_vector():
    # crypto_secretbox test vector from the NaCl distribution (tests/secretbox.c)
    k = bytes.fromhex("1b27556473e985d462cd51197a9a46c76009549eac6474f206c4ee0844f68389")
    n = bytes.fromhex("69696ee955b62b73cd62bda875fc73d68219e0036b7a0b37")
    m = bytes.fromhex("be075fc53c81f2d5cf141316ebeb0c7b5228c52a4c62cbd44b66849b64244ffce5ecbaaf33bd751a1ac728d4"
                      "5e6c61296cdc3c01233561f41db66cce314adb310e3be8250c46f06dceea3a7fa1348057e2f6556ad6b1318a"
                      "024a838f21af1fde048977eb48f59ffd4924ca1c60902e52f0a089bc76897040e082f937763848645e0705")
    c = crypto.secretbox_seal(k, n, m)
    assert c.hex().startswith("f3ffc7703f9400e52a7dfb4b3d3305d98e993b9f48681273c29650ba32fc76ce48332ea7")
    assert c.hex().endswith("a43d14a6599b1f654cb45a74e355a5")
    assert crypto.secretbox_open(k, n, c) == m
    bad = bytearray(c)
    bad[20] ^= 1
    with pytest.raises(crypto.CryptoError):
        crypto.secretbox_open(k, n, bytes(bad))


@pytest.mark.parametrize("kind,size", [("aescbc", 16), ("aescbc", 32), ("aesgcm", 16), ("aesgcm", 32), ("secretbox", 32)])
def test_transformer_roundtrip(kind, size):
    t = v.load_encryption_config(config({kind: {"keys": [{"name": "k1", "secret": b64(size)}]}}))["secrets"]
    for data in (b"", b"x", b"0123456789abcdef", os.urandom(1000)):
        out = t.to_storage(data, b"/registry/secrets/default/s1")
        assert out.startswith(f"k8s:enc:{kind}:v1:k1:".encode())
        assert t.from_storage(out, b"/registry/secrets/default/s1") == (data, False)


def test_gcm_binds_the_key_path():
    t = v.load_encryption_config(config({"aesgcm": {"keys": [{"name": "k1", "secret": b64(32)}]}}))["secrets"]
    out = t.to_storage(b"payload", b"/registry/secrets/default/a")
    with pytest.raises(v.TransformError):
        t.from_storage(out, b"/registry/secrets/default/b")   # copied to another key: rejected


def test_key_rotation_and_stale_reads():
    old = config({"aescbc": {"keys": [{"name": "old", "secret": b64(32, 1)}]}})
    new = config({"aescbc": {"keys": [{"name": "new", "secret": b64(32, 2)}, {"name": "old", "secret": b64(32, 1)}]}})
    t_old = v.load_encryption_config(old)["secrets"]
    t_new = v.load_encryption_config(new)["secrets"]
    stored = t_old.to_storage(b"data", b"k")
    assert t_new.from_storage(stored, b"k") == (b"data", True)     # readable, flagged stale
    assert t_new.to_storage(b"data", b"k").startswith(b"k8s:enc:aescbc:v1:new:")
    # identity first: plaintext writes, encrypted values still readable
    mixed = v.load_encryption_config(config({"identity": {}}, {"aescbc": {"keys": [{"name": "old", "secret": b64(32, 1)}]}}))["secrets"]
    assert mixed.to_storage(b"plain", b"k") == b"plain"
    assert mixed.from_storage(stored, b"k") == (b"data", True)
    assert mixed.from_storage(b'{"a":1}', b"k") == (b'{"a":1}', False)


def test_bad_config_rejected():
    with pytest.raises(v.TransformError):
        v.load_encryption_config({"kind": "Nope"})
    with pytest.raises(v.TransformError):
        v.load_encryption_config(config({"aescbc": {"keys": [{"name": "k", "secret": b64(7)}]}}))


def test_kms_envelope(tmp_path):
    kms = LocalKMS(str(tmp_path / "kms.sock")).start()
    try:
        cfg = config({"kms": {"name": "local", "endpoint": "unix://" + str(tmp_path / "kms.sock"), "cachesize": 10}})
        t = v.load_encryption_config(cfg)["secrets"]
        out = t.to_storage(b"secret-data", b"k")
        assert out.startswith(b"k8s:enc:kms:v1:local:")
        assert b"secret-data" not in out
        assert kms.calls["Encrypt"] == 1
        # a fresh transformer (empty DEK cache) must go to the KMS to unwrap the DEK
        t2 = v.load_encryption_config(cfg)["secrets"]
        assert t2.from_storage(out, b"k") == (b"secret-data", False)
        assert kms.calls["Decrypt"] == 1
        assert t2.from_storage(out, b"k")[0] == b"secret-data"
        assert kms.calls["Decrypt"] == 1                          # cached
        assert KMSClient("unix://" + str(tmp_path / "kms.sock")).version() == ("v1beta1", "kamd-local-kms")
    finally:
        kms.stop()


def _raw(server, key):
    kvs, _, _ = server.store.range(key)
    return kvs[0].value


def test_apiserver_encrypts_secrets_at_rest(run, tmp_path):
    wal = str(tmp_path / "wal")
    cfg = config({"aescbc": {"keys": [{"name": "k1", "secret": b64(32)}]}}, {"identity": {}})

    async def main():
        from kubernetes_amd.storage.mvcc import MVCCStore
        s = APIServer(store=MVCCStore(wal_path=wal), encryption_config=cfg)
        port = await s.start()
        c = Client(f"http://127.0.0.1:{port}")
        try:
            await c.create("secrets", dict(SECRET))
            await c.create("configmaps", {"metadata": {"name": "cm", "namespace": "default"}, "data": {"k": "visible"}})
            raw = _raw(s, "/registry/secrets/default/s1")
            assert raw.startswith(b"k8s:enc:aescbc:v1:k1:")
            assert SECRET["data"]["password"].encode() not in raw
            assert b"visible" in _raw(s, "/registry/configmaps/default/cm")     # not configured: plaintext
            got = await c.get("secrets", "s1", "default")
            assert got["data"] == SECRET["data"]
            got["data"]["extra"] = base64.b64encode(b"more").decode()
            await c.update("secrets", got)
            assert _raw(s, "/registry/secrets/default/s1").startswith(b"k8s:enc:aescbc:v1:k1:")
        finally:
            await c.close()
            await s.stop()
        s.store.close() if hasattr(s.store, "close") else None
        # restart from the WAL: caches are rebuilt by decrypting
        s2 = APIServer(store=MVCCStore(wal_path=wal), encryption_config=cfg)
        assert s2.get_object("secrets", "default", "s1")["data"]["extra"] == base64.b64encode(b"more").decode()
    run(main())


def test_shared_store_workers_encrypt(run):
    cfg = config({"secretbox": {"keys": [{"name": "sb", "secret": b64(32, 3)}]}})
    store = StoreServer()
    addr = store.start()

    async def main():
        a = APIServer(store=addr, encryption_config=cfg)
        b = APIServer(store=addr, encryption_config=cfg)
        pa, pb = await a.start(), await b.start()
        ca, cb = Client(f"http://127.0.0.1:{pa}"), Client(f"http://127.0.0.1:{pb}")
        try:
            await ca.create("secrets", dict(SECRET))
            kv = await a.rstore.get("/registry/secrets/default/s1")
            assert kv.value.startswith(b"k8s:enc:secretbox:v1:sb:")
            assert SECRET["data"]["password"].encode() not in kv.value
            for _ in range(200):
                try:
                    got = await cb.get("secrets", "s1", "default")
                    break
                except Exception:
                    import asyncio
                    await asyncio.sleep(0.01)
            assert got["data"] == SECRET["data"]
            # rbac objects live under "<plural>.<group>" keys: the other worker must see them too
            await ca.create("roles", {"metadata": {"name": "r", "namespace": "default"}, "rules": []})
            import asyncio
            for _ in range(200):
                if b.get_object("roles", "default", "r") is not None:
                    break
                await asyncio.sleep(0.01)
            assert b.get_object("roles", "default", "r") is not None
            await cb.delete("secrets", "s1", "default")
        finally:
            await ca.close()
            await cb.close()
            await a.stop()
            await b.stop()
    try:
        run(main())
    finally:
        store.stop()
