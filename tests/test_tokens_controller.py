"""Service-account tokens controller table cases (`pkg/controller/serviceaccount/
tokens_controller_test.go` TestTokenCreation): an account without a referenced token gets one,
a deleted account's tokens go, a token secret for a missing (or re-created, other-UID) account is
deleted, a token secret missing its token / namespace / CA data is filled in, and deleting a
referenced token secret drops the reference (after which the account gets a fresh token)."""
import asyncio
import base64

from kubernetes_amd.client.fake import FakeClient
from kubernetes_amd.client.informer import InformerFactory
from kubernetes_amd.controllers.certificates import SA_NAME_ANN, SA_TOKEN, SA_UID_ANN, TokensController
from kubernetes_amd.native import crypto

KEY = None


def _key():
    global KEY
    if KEY is None:
        KEY = crypto.generate_key("rsa", 2048)
    return KEY


def sa(name="default", uid="sa-uid", secrets=()):
    return {"apiVersion": "v1", "kind": "ServiceAccount",
            "metadata": {"name": name, "namespace": "default", "uid": uid},
            "secrets": [{"name": s} for s in secrets]}


def token(name, sa_name="default", uid="sa-uid", data=None):
    return {"apiVersion": "v1", "kind": "Secret", "type": SA_TOKEN,
            "metadata": {"name": name, "namespace": "default",
                         "annotations": {SA_NAME_ANN: sa_name, SA_UID_ANN: uid}},
            "data": data if data is not None else {"token": "dG9r", "namespace": "ZGVmYXVsdA==",
                                                     "ca.crt": base64.b64encode(b"CA").decode()}}


def run(*objs, keys=(), act=None):
    async def main():
        c = FakeClient(*objs)
        f = InformerFactory(c)
        ctl = TokensController(c, f, private_key=_key(), root_ca="CA")
        ctl.setup()
        f.start()
        await f.wait_for_cache_sync()
        if act:
            await act(c, ctl)
            await asyncio.sleep(0.05)
        for k in keys:
            await ctl.sync(k)
            await asyncio.sleep(0.05)
        return c
    return asyncio.run(main())


def secrets(c):
    return {k[1]: v for k, v in c.objects.get("secrets", {}).items()}


def account(c, name="default"):
    return c.objects["serviceaccounts"][("default", name)]


def test_new_account_gets_a_referenced_token():
    c = run(sa(), keys=["sa:default/default"])
    (name, sec), = secrets(c).items()
    assert name.startswith("default-token-") and sec["type"] == SA_TOKEN
    assert sec["metadata"]["annotations"][SA_UID_ANN] == "sa-uid"
    assert base64.b64decode(sec["data"]["ca.crt"]).decode() == "CA"
    assert [r["name"] for r in account(c)["secrets"]] == [name]


def test_account_with_a_referenced_token_is_left_alone():
    c = run(sa(secrets=["t1"]), token("t1"), keys=["sa:default/default"])
    assert list(secrets(c)) == ["t1"] and [r["name"] for r in account(c)["secrets"]] == ["t1"]


def test_account_referencing_a_missing_or_non_token_secret_gets_a_token():
    plain = {"apiVersion": "v1", "kind": "Secret", "metadata": {"name": "regular", "namespace": "default"}}
    c = run(sa(secrets=["regular", "gone"]), plain, keys=["sa:default/default"])
    new = [n for n in secrets(c) if n.startswith("default-token-")]
    assert len(new) == 1
    assert [r["name"] for r in account(c)["secrets"]] == ["regular", "gone", new[0]]


def test_unreferenced_existing_token_is_referenced_not_duplicated():
    c = run(sa(), token("t1"), keys=["sa:default/default"])
    assert list(secrets(c)) == ["t1"] and [r["name"] for r in account(c)["secrets"]] == ["t1"]


def test_deleted_account_tokens_are_deleted():
    c = run(token("t1"), token("t2"), token("other", sa_name="builder"), keys=["sa:default/default"])
    assert list(secrets(c)) == ["other"]


def test_token_for_missing_or_recreated_account_is_deleted():
    c = run(token("t1"), keys=["secret:default/t1"])
    assert secrets(c) == {}
    c = run(sa(uid="new-uid"), token("t1", uid="old-uid"), keys=["secret:default/t1"])
    assert secrets(c) == {}
    c = run(sa(), token("t1"), keys=["secret:default/t1"])
    assert list(secrets(c)) == ["t1"]


def test_token_secret_missing_data_is_filled_in():
    c = run(sa(secrets=["t1"]), token("t1", data={}), keys=["secret:default/t1"])
    d = secrets(c)["t1"]["data"]
    assert d["token"] and base64.b64decode(d["namespace"]).decode() == "default"
    assert base64.b64decode(d["ca.crt"]).decode() == "CA"
    # only the CA is stale: the token itself is kept
    c = run(sa(secrets=["t1"]), token("t1", data={"token": "dG9r", "namespace": "ZGVmYXVsdA==",
                                                   "ca.crt": "b2xk"}), keys=["secret:default/t1"])
    d = secrets(c)["t1"]["data"]
    assert d["token"] == "dG9r" and base64.b64decode(d["ca.crt"]).decode() == "CA"


def test_deleting_a_referenced_token_drops_the_reference_and_reissues():
    async def delete(c, ctl):
        await c.delete("secrets", "t1", "default")
    c = run(sa(secrets=["t1", "regular"]), token("t1"), act=delete, keys=["secret:default/t1", "sa:default/default"])
    refs = [r["name"] for r in account(c)["secrets"]]
    assert "t1" not in refs and refs[0] == "regular"
    new = [n for n in secrets(c) if n.startswith("default-token-")]
    assert len(new) == 1 and refs == ["regular", new[0]]
