"""`kubectl create configmap|secret --append-hash`, ported from `pkg/kubectl/util/hash/hash_test.go`
(TestConfigMapHash, TestSecretHash, TestEncodeConfigMap, TestEncodeSecret) — the hashes are the
reference's literal expected values."""
import base64

import pytest

from kubernetes_amd.kubectl.extra import generate
from kubernetes_amd.kubectl.hash import config_map_hash, encode_config_map, encode_hash, encode_secret, secret_hash


def b(s):
    return base64.b64encode(s.encode()).decode()


@pytest.mark.parametrize("data,want,enc", [
    ({}, "42745tchd9", '{"data":{},"kind":"ConfigMap","name":""}'),
    ({"one": ""}, "9g67k2htb6", '{"data":{"one":""},"kind":"ConfigMap","name":""}'),
    ({"two": "2", "one": "", "three": "3"}, "f5h7t85m9b", '{"data":{"one":"","three":"3","two":"2"},"kind":"ConfigMap","name":""}'),
])
def test_config_map_hash(data, want, enc):
    cm = {"data": data}
    assert config_map_hash(cm) == want and encode_config_map(cm) == enc


@pytest.mark.parametrize("data,want,enc", [
    ({}, "t75bgf6ctb", '{"data":{},"kind":"Secret","name":"","type":"my-type"}'),
    ({"one": b("")}, "74bd68bm66", '{"data":{"one":""},"kind":"Secret","name":"","type":"my-type"}'),
    ({"two": b("2"), "one": b(""), "three": b("3")}, "dgcb6h9tmk",
     '{"data":{"one":"","three":"Mw==","two":"Mg=="},"kind":"Secret","name":"","type":"my-type"}'),
])
def test_secret_hash(data, want, enc):
    sec = {"type": "my-type", "data": data}
    assert secret_hash(sec) == want and encode_secret(sec) == enc


def test_encode_hash():
    assert encode_hash("0123456789abcdef") == "gh2k456789" and encode_hash("aaeeaaeeaa") == "mmttmmttmm"
    with pytest.raises(ValueError):
        encode_hash("123")


def test_create_with_append_hash():
    plural, cm = generate(["configmap", "app", "--from-literal=a=1", "--append-hash"], "default")
    assert plural == "configmaps"
    assert cm["metadata"]["name"] == "app-" + config_map_hash({"metadata": {"name": "app"}, "data": {"a": "1"}})
    plural, sec = generate(["secret", "generic", "s", "--from-literal=k=v", "--append-hash"], "default")
    assert sec["metadata"]["name"] == "s-" + secret_hash({"metadata": {"name": "s"}, "type": "Opaque",
                                                         "data": {"k": b("v")}})
    _, plain = generate(["configmap", "app", "--from-literal=a=1"], "default")
    assert plain["metadata"]["name"] == "app"
