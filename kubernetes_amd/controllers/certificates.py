"""Identity controllers: service-account tokens, bootstrap signer / token cleaner, CSR approving
and signing, cluster-role aggregation, node TTL.

Parity:
  * `pkg/controller/serviceaccount/tokens_controller.go` — every ServiceAccount gets a
    `kubernetes.io/service-account-token` secret `<sa>-token-<5 chars>` holding a signed JWT,
    `ca.crt` and `namespace`, annotated with the SA name/uid and referenced from `sa.secrets`;
    token secrets whose SA is gone are deleted;
  * `pkg/controller/bootstrap/bootstrapsigner.go` — `kube-public/cluster-info` gets a detached
    JWS (`<b64 header>..<b64 HMAC-SHA256>`, key = `<id>.<secret>`) per signing bootstrap token
    under `jws-kubeconfig-<id>`; `tokencleaner.go` deletes expired bootstrap token secrets;
  * `pkg/controller/certificates/approver/sarapprove.go:82-229` — auto-approve node client
    CSRs (O=system:nodes, CN=system:node:*, usages exactly {key encipherment, digital signature,
    client auth}) when a SubjectAccessReview allows `create certificatesigningrequests/nodeclient`
    (or `/selfnodeclient` when the requester is the node itself);
  * `pkg/controller/certificates/signer/cfssl_signer.go` — approved CSRs are signed by the
    cluster CA (`--cluster-signing-cert-file/--cluster-signing-key-file`, 1 year);
  * `pkg/controller/clusterroleaggregation` — `aggregationRule.clusterRoleSelectors` -> rules;
  * `pkg/controller/ttl/ttl_controller.go` — node annotation `node.alpha.kubernetes.io/ttl`
    from cluster size (0 s up to 100 nodes, 15 s to 500, 30 s to 1000, 60 s to 2000, 300 s beyond).
"""
from __future__ import annotations

import asyncio
import base64
import hashlib
import hmac
import json
import random
import time

from ..api import meta as m
from ..api.labels import label_selector_as_selector
from ..api.meta import parse_rfc3339
from ..client.rest import APIStatusError, is_already_exists, is_not_found
from .base import Controller, split_key

SA_TOKEN = "kubernetes.io/service-account-token"
SA_NAME_ANN = "kubernetes.io/service-account.name"
SA_UID_ANN = "kubernetes.io/service-account.uid"
BOOTSTRAP = "bootstrap.kubernetes.io/token"


def _b64(v: str) -> str:
    return base64.b64encode(v.encode()).decode()


def _sdata(sec, k):
    v = (sec.get("data") or {}).get(k)
    try:
        return base64.b64decode(v).decode() if v is not None else None
    except Exception:
        return None


class TokensController(Controller):
    name = "serviceaccount-token"
    workers = 2

    def __init__(self, client, factory, private_key=None, private_key_file=None, root_ca=None, root_ca_file=None, **kw):
        super().__init__(client, factory, **kw)
        if private_key_file:
            with open(private_key_file) as f:
                private_key = f.read()
        if root_ca_file:
            with open(root_ca_file) as f:
                root_ca = f.read()
        self.key = private_key
        self.root_ca = root_ca or ""
        self._deleted_refs: dict = {}          # deleted token secret -> (account name, account uid)

    def setup(self):
        self.sa_inf = self.factory.get("serviceaccounts")
        self.sec_inf = self.factory.get("secrets")
        self.sa_inf.add_handler(self._sa, lambda o, n: self._sa(n), self._sa)
        self.sec_inf.add_handler(self._secret, lambda o, n: self._secret(n), self._secret_deleted)

    def _sa(self, sa):
        self.queue.add("sa:" + m.ns_name(sa))

    def _secret(self, sec):
        if sec.get("type") == SA_TOKEN:
            self.queue.add("secret:" + m.ns_name(sec))

    def _secret_deleted(self, sec):
        """`deleteSecret`: the service account must stop referencing it."""
        if sec.get("type") == SA_TOKEN:
            ann = sec["metadata"].get("annotations") or {}
            self._deleted_refs[m.ns_name(sec)] = (ann.get(SA_NAME_ANN, ""), ann.get(SA_UID_ANN, ""))
            self.queue.add("secret:" + m.ns_name(sec))

    def _tokens_of(self, ns, name, uid):
        return [s for s in self.sec_inf.list() if s.get("type") == SA_TOKEN and s["metadata"].get("namespace") == ns
                and (s["metadata"].get("annotations") or {}).get(SA_NAME_ANN) == name]

    def resync_keys(self):
        return ["sa:" + m.ns_name(sa) for sa in self.sa_inf.list()]

    async def sync(self, key):
        if not self.key:
            return
        kind, _, k = key.partition(":")
        if kind == "secret":
            await self.sync_secret(k)
        else:
            await self.sync_service_account(k if kind == "sa" else key)

    def _token_data(self, sa, ns, secret_name):
        from ..apiserver.authn import service_account_token
        return {"token": _b64(service_account_token(self.key, sa, secret_name)), "namespace": _b64(ns),
                "ca.crt": _b64(self.root_ca)}

    async def sync_service_account(self, key):
        """`syncServiceAccount`: a deleted account's tokens are deleted; a live one gets a token
        secret if it references none (`ensureReferencedToken`)."""
        ns, name = split_key(key)
        sa = self.sa_inf.get(key)
        toks = self._tokens_of(ns, name, None)
        if sa is None:
            for t in toks:     # SA deleted: its tokens go
                try:
                    await self.client.delete("secrets", t["metadata"]["name"], ns)
                except APIStatusError as e:
                    if not is_not_found(e):
                        raise
            return
        uid = sa["metadata"].get("uid", "")
        live = [t for t in toks if (t["metadata"].get("annotations") or {}).get(SA_UID_ANN) == uid]
        refs = [r.get("name") for r in sa.get("secrets") or ()]
        if any(t["metadata"]["name"] in refs for t in live):
            return                 # hasReferencedToken
        if not live:
            sname = f"{name}-token-{''.join(random.choice('bcdfghjklmnpqrstvwxz2456789') for _ in range(5))}"
            sec = {"metadata": {"name": sname, "namespace": ns, "annotations": {SA_NAME_ANN: name, SA_UID_ANN: uid}},
                   "type": SA_TOKEN, "data": self._token_data(sa, ns, sname)}
            try:
                await self.client.create("secrets", sec, ns)
            except APIStatusError as e:
                if not is_already_exists(e):
                    raise
            live = [sec]
        want = refs + [t["metadata"]["name"] for t in live if t["metadata"]["name"] not in refs]
        if want != refs:
            # an update of the live object (`tokens_controller.go` ensureReferencedToken): the
            # system:kube-controller-manager role may update service accounts, not patch them;
            # a conflict re-queues the key
            live_sa = await self.client.get("serviceaccounts", name, ns)
            have = [r.get("name") for r in live_sa.get("secrets") or ()]
            add = [n for n in want if n not in have]
            if add:
                live_sa["secrets"] = (live_sa.get("secrets") or []) + [{"name": n} for n in add]
                await self.client.update("serviceaccounts", live_sa, ns)

    async def sync_secret(self, key):
        """`syncSecret`: a deleted token secret is removed from its account's references; a token
        secret whose account is gone (or is another account by UID) is deleted; one missing its
        token, namespace or CA data gets them (`generateTokenIfNeeded`)."""
        ns, name = split_key(key)
        sec = self.sec_inf.get(key)
        if sec is None:
            sa_name, sa_uid = self._deleted_refs.pop(key, ("", ""))
            sa = self.sa_inf.get(f"{ns}/{sa_name}") if sa_name else None
            if sa is None or (sa_uid and sa["metadata"].get("uid") != sa_uid):
                return
            if any(r.get("name") == name for r in sa.get("secrets") or ()):
                live_sa = await self.client.get("serviceaccounts", sa_name, ns)
                live_sa["secrets"] = [r for r in live_sa.get("secrets") or () if r.get("name") != name]
                await self.client.update("serviceaccounts", live_sa, ns)
            self.queue.add(f"sa:{ns}/{sa_name}")       # it may need a new token
            return
        ann = sec["metadata"].get("annotations") or {}
        sa = self.sa_inf.get(f"{ns}/{ann.get(SA_NAME_ANN, '')}")
        if sa is None or (ann.get(SA_UID_ANN) and sa["metadata"].get("uid") != ann.get(SA_UID_ANN)):
            try:
                await self.client.delete("secrets", name, ns)
            except APIStatusError as e:
                if not is_not_found(e):
                    raise
            return
        data = sec.get("data") or {}
        want_ns, want_ca = _b64(ns), _b64(self.root_ca)
        needs = (not data.get("token"), data.get("namespace") != want_ns, bool(self.root_ca) and data.get("ca.crt") != want_ca)
        if not any(needs):
            return
        live = await self.client.get("secrets", name, ns)
        d = dict(live.get("data") or {})
        if needs[0]:
            d["token"] = self._token_data(sa, ns, name)["token"]
        d["namespace"] = want_ns
        if self.root_ca:
            d["ca.crt"] = want_ca
        live["data"] = d
        await self.client.update("secrets", live, ns)


def jws_detached(token_id, token_secret, payload: str) -> str:
    header = base64.urlsafe_b64encode(json.dumps({"alg": "HS256", "kid": token_id}, separators=(",", ":")).encode()).rstrip(b"=")
    body = base64.urlsafe_b64encode(payload.encode()).rstrip(b"=")
    sig = hmac.new(f"{token_id}.{token_secret}".encode(), header + b"." + body, hashlib.sha256).digest()
    return (header + b".." + base64.urlsafe_b64encode(sig).rstrip(b"=")).decode()


class BootstrapSignerController(Controller):
    name = "bootstrapsigner"
    workers = 1

    def setup(self):
        self.cm_inf = self.factory.get("configmaps", "kube-public")
        self.sec_inf = self.factory.get("secrets", "kube-system")
        self.cm_inf.add_handler(lambda o: self.enqueue("kube-public/cluster-info"), lambda o, n: self.enqueue("kube-public/cluster-info"), None)
        self.sec_inf.add_handler(lambda o: self.enqueue("kube-public/cluster-info"),
                                 lambda o, n: self.enqueue("kube-public/cluster-info"),
                                 lambda o: self.enqueue("kube-public/cluster-info"))

    async def sync(self, key):
        cm = self.cm_inf.get("kube-public/cluster-info")
        if cm is None:
            return
        kc = (cm.get("data") or {}).get("kubeconfig")
        if kc is None:
            return
        sigs = {}
        now = time.time()
        for s in self.sec_inf.list():
            if s.get("type") != BOOTSTRAP or _sdata(s, "usage-bootstrap-signing") != "true":
                continue
            exp = _sdata(s, "expiration")
            if exp and (parse_rfc3339(exp) or 0) < now:
                continue
            tid, tsec = _sdata(s, "token-id"), _sdata(s, "token-secret")
            if tid and tsec:
                sigs[f"jws-kubeconfig-{tid}"] = jws_detached(tid, tsec, kc)
        data = {k: v for k, v in (cm.get("data") or {}).items() if not k.startswith("jws-kubeconfig-")}
        data.update(sigs)
        if data != cm.get("data"):
            cm = dict(cm, data=data)
            await self.client.update("configmaps", cm, "kube-public")


class TokenCleanerController(Controller):
    name = "tokencleaner"
    workers = 1

    def setup(self):
        self.sec_inf = self.factory.get("secrets", "kube-system")
        self.sec_inf.add_handler(self.enqueue, lambda o, n: self.enqueue(n), None)
        self._tick = None

    def start(self):
        super().start()
        self._tick = asyncio.ensure_future(self._ticker())

    def stop(self):
        super().stop()
        if self._tick:
            self._tick.cancel()

    async def _ticker(self):
        while True:
            await asyncio.sleep(5)
            for s in self.sec_inf.list():
                if s.get("type") == BOOTSTRAP:
                    self.enqueue(s)

    async def sync(self, key):
        s = self.sec_inf.get(key)
        if s is None or s.get("type") != BOOTSTRAP:
            return
        exp = _sdata(s, "expiration")
        if exp and (parse_rfc3339(exp) or 0) < time.time():
            ns, name = split_key(key)
            try:
                await self.client.delete("secrets", name, ns)
            except APIStatusError as e:
                if not is_not_found(e):
                    raise


KUBELET_CLIENT_USAGES = {"key encipherment", "digital signature", "client auth"}


def _approval(csr):
    for c in (csr.get("status") or {}).get("conditions") or ():
        if c.get("type") in ("Approved", "Denied"):
            return c["type"]
    return None


def _csr_pem(csr):
    return base64.b64decode((csr.get("spec") or {}).get("request", "")).decode()


class CSRApprovingController(Controller):
    name = "csrapproving"
    workers = 1

    def setup(self):
        self.csr_inf = self.factory.get("certificatesigningrequests")
        self.csr_inf.add_handler(self.enqueue, lambda o, n: self.enqueue(n), None)

    async def sync(self, key):
        from ..native import crypto
        csr = self.csr_inf.get(key)
        if csr is None or (csr.get("status") or {}).get("certificate") or _approval(csr):
            return
        sp = csr.get("spec") or {}
        try:
            cn, orgs = crypto.csr_subject(_csr_pem(csr))
        except Exception:
            return
        if orgs != ["system:nodes"] or not cn.startswith("system:node:") or set(sp.get("usages") or ()) != KUBELET_CLIENT_USAGES \
                or len(sp.get("usages") or ()) != 3:
            return
        sub = "selfnodeclient" if sp.get("username") == cn else "nodeclient"
        sar = await self.client.create("subjectaccessreviews", {"spec": {
            "user": sp.get("username", ""), "uid": sp.get("uid", ""), "groups": sp.get("groups") or [],
            "resourceAttributes": {"group": "certificates.k8s.io", "resource": "certificatesigningrequests",
                                   "verb": "create", "subresource": sub}}})
        if not (sar.get("status") or {}).get("allowed"):
            return
        csr = dict(csr)
        st = dict(csr.get("status") or {})
        st["conditions"] = list(st.get("conditions") or []) + [
            {"type": "Approved", "reason": "AutoApproved",
             "message": "Auto approving self kubelet client certificate after SubjectAccessReview." if sub == "selfnodeclient"
             else "Auto approving kubelet client certificate after SubjectAccessReview."}]
        csr["status"] = st
        await self.client.update("certificatesigningrequests", csr, subresource="approval")


class CSRSigningController(Controller):
    name = "csrsigning"
    workers = 1

    def __init__(self, client, factory, ca_cert=None, ca_key=None, cert_file=None, key_file=None, days=365, **kw):
        super().__init__(client, factory, **kw)
        if cert_file:
            with open(cert_file) as f:
                ca_cert = f.read()
        if key_file:
            with open(key_file) as f:
                ca_key = f.read()
        self.ca_cert, self.ca_key, self.days = ca_cert, ca_key, days

    def setup(self):
        self.csr_inf = self.factory.get("certificatesigningrequests")
        self.csr_inf.add_handler(self.enqueue, lambda o, n: self.enqueue(n), None)

    async def sync(self, key):
        from ..native import crypto
        csr = self.csr_inf.get(key)
        if not self.ca_cert or csr is None or (csr.get("status") or {}).get("certificate") or _approval(csr) != "Approved":
            return
        usages = set((csr.get("spec") or {}).get("usages") or ())
        usage = "client" if "server auth" not in usages else ("server" if "client auth" not in usages else "both")
        cert = crypto.issue_cert(csr_pem=_csr_pem(csr), ca_cert=self.ca_cert, ca_key=self.ca_key, days=self.days, usage=usage)
        csr = dict(csr)
        csr["status"] = dict(csr.get("status") or {}, certificate=base64.b64encode(cert.encode()).decode())
        await self.client.update_status("certificatesigningrequests", csr)


class CSRCleanerController(Controller):
    """`pkg/controller/certificates/cleaner/cleaner.go`: every pollingInterval (1 h) each CSR is
    deleted when it was approved and issued more than an hour ago, denied more than an hour ago,
    left unhandled (no conditions) for a day, or carries an issued certificate that has expired."""
    name = "csrcleaner"
    workers = 1
    resync_period = 3600.0          # pollingInterval
    APPROVED_EXPIRATION = 3600.0
    DENIED_EXPIRATION = 3600.0
    PENDING_EXPIRATION = 24 * 3600.0

    primary = "certificatesigningrequests"

    def setup(self):
        self.csr_inf = self.factory.get("certificatesigningrequests")
        self.csr_inf.add_handler(self.enqueue, None, None)      # the initial list: wait.Until runs at once

    @classmethod
    def should_clean(cls, csr, now=None):
        now = time.time() if now is None else now

        def older(ts, d):
            t = parse_rfc3339(ts) if ts else None
            return t is not None and t < now - d
        conds = (csr.get("status") or {}).get("conditions") or []
        cert = (csr.get("status") or {}).get("certificate")
        if not conds and older(csr["metadata"].get("creationTimestamp"), cls.PENDING_EXPIRATION):
            return "pending"
        for c in conds:
            if c.get("type") == "Denied" and older(c.get("lastUpdateTime"), cls.DENIED_EXPIRATION):
                return "denied"
            if c.get("type") == "Approved" and cert:
                if older(c.get("lastUpdateTime"), cls.APPROVED_EXPIRATION):
                    return "approved"
                from ..native import crypto
                try:
                    if crypto.cert_not_after(base64.b64decode(cert).decode()) < now:
                        return "expired"
                except Exception:      # noqa: BLE001 - `isExpired`: an unparsable certificate is an error, not a clean
                    return None
        return None

    async def sync(self, key):
        csr = self.csr_inf.get(key)
        if csr is None or not self.should_clean(csr):
            return
        try:
            await self.client.delete("certificatesigningrequests", key)
        except APIStatusError as e:
            if not is_not_found(e):
                raise


class ClusterRoleAggregationController(Controller):
    name = "clusterroleaggregation"
    workers = 1

    def setup(self):
        self.cr_inf = self.factory.get("clusterroles")
        self.cr_inf.add_handler(self._any, lambda o, n: self._any(n), self._any)

    def _any(self, _):
        for cr in self.cr_inf.list():
            if cr.get("aggregationRule"):
                self.enqueue(cr)

    async def sync(self, key):
        cr = self.cr_inf.get(key)
        if cr is None or not cr.get("aggregationRule"):
            return
        rules = []
        sels = [label_selector_as_selector(s) for s in cr["aggregationRule"].get("clusterRoleSelectors") or ()]
        for other in sorted(self.cr_inf.list(), key=lambda o: o["metadata"]["name"]):
            if other["metadata"]["name"] == cr["metadata"]["name"]:
                continue
            if any(s.matches(other["metadata"].get("labels") or {}) for s in sels):
                for r in other.get("rules") or ():
                    if r not in rules:
                        rules.append(r)
        if rules != (cr.get("rules") or []):
            await self.client.update("clusterroles", dict(cr, rules=rules))


TTL_ANN = "node.alpha.kubernetes.io/ttl"
# `ttl_controller.go` ttlBoundaries: (sizeMin, sizeMax, ttlSeconds); the overlapping ranges are
# the hysteresis that keeps a cluster near a boundary from flapping
TTL_BOUNDARIES = ((0, 100, 0), (90, 500, 15), (450, 1000, 30), (900, 2000, 60), (1800, 10000, 300),
                  (9000, 2 ** 31 - 1, 600))


def ttl_for(n):
    """The TTL a cluster grown node by node from zero to n nodes settles on."""
    step = 0
    while n > TTL_BOUNDARIES[step][1]:
        step += 1
    return TTL_BOUNDARIES[step][2]


class TTLController(Controller):
    """`pkg/controller/ttl/ttl_controller.go`: every node carries
    `node.alpha.kubernetes.io/ttl` — how long a kubelet may cache secrets/configmaps — set from
    the cluster size; node adds move the boundary step up past sizeMax, deletes move it down
    below sizeMin (hysteresis), and a node is patched when its annotation differs."""
    name = "ttl"
    workers = 1

    def setup(self):
        self.node_inf = self.factory.get("nodes")
        self.node_count = 0
        self.step = 0
        self.node_inf.add_handler(self._add, lambda o, n: self.enqueue(n), self._delete)

    @property
    def desired_ttl(self):
        return TTL_BOUNDARIES[self.step][2]

    def _add(self, node):
        self.node_count += 1
        if self.node_count > TTL_BOUNDARIES[self.step][1]:
            self.step += 1
        self.enqueue(node)

    def _delete(self, node):
        self.node_count -= 1
        if self.step > 0 and self.node_count < TTL_BOUNDARIES[self.step][0]:
            self.step -= 1

    async def sync(self, key):
        node = self.node_inf.get(key)
        if node is None:
            return
        want = str(self.desired_ttl)
        if (node["metadata"].get("annotations") or {}).get(TTL_ANN) != want:
            await self.client.patch("nodes", key, {"metadata": {"annotations": {TTL_ANN: want}}})
