"""kube-apiserver equivalent: REST + watch over HTTP/1.1 on an embedded MVCC store.

Parity map:
  * handler chain (`staging/src/k8s.io/apiserver/pkg/server/config.go:530-551`): panic
    recovery → request info → authentication → max-in-flight → authorization → handler.
  * create/update/patch/delete/list/watch handlers (`staging/src/k8s.io/apiserver/pkg/endpoints/handlers/*.go`),
    mutating admission before validation, validating admission after
    (`handlers/create.go:80-111`).
  * `pods/binding` (fork F6) and `/bindings`, `pods/status`, `nodes/status`,
    `namespaces/{ns}/finalize`, `pods/eviction`, `pods/log` (proxied to the kubelet).
  * discovery (`/api`, `/apis`, `/api/v1`, `/apis/<g>/<v>`), `/healthz`, `/version`, `/metrics`.

Two storage modes:
  * embedded (default): the MVCC store lives in this process; every write is committed and
    dispatched to watchers synchronously on the event loop, so a watcher can never observe
    revisions out of order and reads are always consistent with the last write.
  * shared (`store="unix:///…"` / `"tcp://…"`): several API server worker processes share
    one native `kamd-etcd` (like several kube-apiservers share etcd). A worker commits with a
    compare-and-swap transaction, the store injects the revision into the encoded object, and
    every worker's watch cache is fed ONLY from the store's ordered watch stream — a write is
    acknowledged once this worker's cache has applied its revision (read-your-writes). Device
    assignments are claimed with per-device keys in the same transaction, so no two pods can
    be bound to one GPU even when the binds race through different workers. A stale cache
    shows up as a failed compare; the request is re-run once the cache caught up.
    High-churn resources (pods, events) are NOT cached by shared-mode workers: their reads go
    to the store (GET/RANGE), their watches to the store's native fan-out, and the worker's
    store watch excludes them — so a worker's CPU per pod does not grow with the number of
    workers (each worker ingesting every pod event capped multi-worker scaling).
"""
from __future__ import annotations

import asyncio
import os
import base64
import logging
import secrets
import time

from ..api import codec, core, defaults, meta as m
from ..api import protobuf as pb
from ..api.labels import SelectorError, parse as parse_labels, parse_field_selector
from ..api.meta import parse_rfc3339, fast_copy, now_rfc3339
from ..api.sharding import QUERY_PARAM, SHARD_OFFSET_LABEL, parse_shard, shard_matches
from ..storage import wire
from ..storage.mvcc import CompactedError, MVCCStore
from ..utils.httpserver import HandoffResponse, HTTPServer, Response, StreamResponse, UpgradeResponse
from ..utils.metrics import Registry
from ..utils.patch import JSONPatchError, apply_patch
from . import impersonation
from . import admission as adm
from .auth import ANONYMOUS, AttributesRecord, TokenAuthenticator, User, build_authorizer
from .cacher import ADDED, DELETED, MODIFIED, Entry, GoneError, ResourceCache, error_event, event_bytes, pb_event_bytes
from .registry import (APIError, already_exists, apply_binding, bad_request, conflict, deletion_stamp,
                       init_object_meta, invalid, not_found, strategy_for)

log = logging.getLogger("apiserver")

def _build_info():
    """gitCommit / gitTreeState / buildDate of `version.Info` (pkg/version/base.go), from the
    package's git checkout when there is one."""
    import subprocess
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    commit, state = "", "unknown"
    try:
        commit = subprocess.run(["git", "-C", here, "rev-parse", "HEAD"], capture_output=True, text=True,
                                timeout=5).stdout.strip()
        dirty = subprocess.run(["git", "-C", here, "status", "--porcelain", "--untracked-files=no"],
                               capture_output=True, text=True, timeout=5).stdout.strip()
        state = "dirty" if dirty else "clean" if commit else "unknown"
    except (OSError, subprocess.SubprocessError):
        pass
    built = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(os.path.getmtime(__file__)))
    return {"gitCommit": commit or "unknown", "gitTreeState": state, "buildDate": built}


VERSION = {"major": "1", "minor": "9", "gitVersion": "v1.9.0-amd.0", **_build_info(), "platform": "linux/amd64",
           "goVersion": "n/a", "compiler": "cpython"}

_READ_VERBS = {"GET": "get", "HEAD": "get"}


def _body(req):
    """The request body as an object: decoded from protobuf already, or JSON."""
    return req.obj if req.obj is not None else codec.loads(req.body)


def _log_container(pod, container):
    """`pkg/registry/core/pod/rest/log.go` validateContainer: the only container when none is
    named, else the name must be one of the pod's (init) containers."""
    spec = pod.get("spec") or {}
    names = [c.get("name") for c in spec.get("containers") or ()]
    init = [c.get("name") for c in spec.get("initContainers") or ()]
    name = pod["metadata"].get("name")
    if not container:
        if len(names) == 1:
            return names[0]
        msg = f"a container name must be specified for pod {name}, choose one of: [{' '.join(names)}]"
        if init:
            msg += f" or one of the init containers: [{' '.join(init)}]"
        raise bad_request(msg)
    if container not in names and container not in init:
        raise bad_request(f"container {container} is not valid for pod {name}")
    return container


def _entry_resp(req, ri, status, e):
    """A cached object as the response body: its protobuf envelope when the client negotiated
    protobuf (no JSON made or parsed), else its JSON bytes."""
    if req.served_gv is None and codec.PROTOBUF in req.headers.get("accept", "") and \
            "as=Table" not in req.headers.get("accept", "") and pb.supported(ri.kind, ri.group_version):
        return Response(status, e.pb_envelope(), codec.PROTOBUF)
    return Response(status, e.raw, entry=e)


def _json(status, obj):
    return Response(status, codec.dumpb(obj))


def _err(e: APIError):
    return Response(e.code, codec.dumpb(m.status_obj(e.code, e.reason, e.message, e.details)))


class _Stale(Exception):
    """Shared-store compare failed: this worker's cache is behind revision `rev`."""

    def __init__(self, rev):
        super().__init__(rev)
        self.rev = rev


# the insecure port's user (`insecure_handler.go`: no authentication, no authorization)
UNSECURED = User("system:unsecured", "", ["system:masters", "system:authenticated"])
SWAGGER_UI_PAGE = (b"<!DOCTYPE html><html><head><title>kube-apiserver API</title></head><body>"
                   b"<h1>kube-apiserver</h1><p>OpenAPI: <a href=\"/swagger.json\">/swagger.json</a> "
                   b"(<a href=\"/openapi/v2\">/openapi/v2</a>)</p></body></html>")


_TIMEOUT_RESPONSE = Response(504, codec.dumpb({"kind": "Status", "apiVersion": "v1", "metadata": {}, "status": "Failure",
                                              "message": "Timeout: request did not complete within allowed duration",
                                              "reason": "Timeout", "details": {}, "code": 504}))


def node_address(node, preferred=("InternalIP", "ExternalIP", "Hostname")):
    """`--kubelet-preferred-address-types`: the first node address of the first listed type."""
    addrs = ((node or {}).get("status") or {}).get("addresses") or ()
    for t in preferred:
        for a in addrs:
            if a.get("type") == t and a.get("address"):
                return a["address"]
    return "127.0.0.1"


def parse_runtime_config(spec):
    """`--runtime-config` (`pkg/master/master.go` DefaultAPIResourceConfigSource + overrides):
    `api/all=false`, `api/legacy=false` (core v1), `<group>/<version>=false|true`,
    `extensions/v1beta1/<resource>=false`; a bare key means true. -> (disabled {(group, version)},
    disabled {(group, version, resource)})."""
    if isinstance(spec, dict):
        items = list(spec.items())
    else:
        items = []
        for part in (spec or "").split(","):
            part = part.strip()
            if part:
                k, _, v = part.partition("=")
                items.append((k, v or "true"))
    all_gv = {(g, v) for g, vs in m.served_versions().items() for v in vs}
    disabled, disabled_res = set(), set()
    for k, v in items:
        on = str(v).lower() in ("true", "1", "")
        if k in ("api/all", "api/*"):
            disabled = set() if on else set(all_gv)
            continue
        if k in ("api/legacy", "api/v1", "v1"):
            gvs = {("", "v1")}
        else:
            bits = k.split("/")
            if len(bits) == 3:
                (disabled_res.discard if on else disabled_res.add)((bits[0], bits[1], bits[2]))
                continue
            if len(bits) != 2:
                raise ValueError(f"invalid --runtime-config key {k!r}")
            gvs = {(bits[0], bits[1])}
        disabled = (disabled - gvs) if on else (disabled | gvs)
    return disabled, disabled_res


def q_include(req):
    return (req.query.get("includeObject") or "Metadata") if hasattr(req, "query") else "Metadata"


class _Missing(Exception):
    """Shared-store cache miss: the object may exist in the store already (this worker lags)."""

    def __init__(self, key, error):
        super().__init__(key)
        self.key, self.error = key, error


def _run_sync(coro):
    """Drive a coroutine that never suspends (embedded-store commit path) to completion."""
    try:
        coro.send(None)
    except StopIteration as e:
        return e.value
    coro.close()
    raise RuntimeError("embedded-store operation suspended")


DEVICE_PREFIX = "/kamd/devices/"   # claim keys, outside /registry/ so watch caches never see them
ENC_PREFIX = b"k8s:enc:"          # encrypted-at-rest value (storage/value.py)
_FRAME = b"\x00KH"                 # shared-store value framing (index header + object)


def pb_to_json(body, rev) -> bytes:
    """A protobuf-stored object (k8s\\0 envelope) as JSON bytes with resourceVersion = rev."""
    return pb.to_json(body, rev)


def _requested_gv(path):
    parts = path.split("/", 4)
    if len(parts) > 2 and parts[1] == "api":
        return parts[2]
    if len(parts) > 3 and parts[1] == "apis":
        return f"{parts[2]}/{parts[3]}"
    return ""


def _rewrite_gv(body, canonical, served):
    """apiVersion of an object / list (and its items) → the version the client asked for."""
    try:
        o = codec.loads(body)
    except ValueError:
        return body
    if o.get("apiVersion") == canonical:
        o["apiVersion"] = served
    for it in o.get("items") or ():
        if isinstance(it, dict) and it.get("apiVersion") in (canonical, None):
            it["apiVersion"] = served
    return codec.dumpb(o)

class APIServer:
    def __init__(self, store=None, admission_plugins=None, admission_config=None, token_file=None, etcd_tls=None,
                 tokens=None, authorization_modes=("AlwaysAllow",), max_requests_inflight=4000,
                 max_mutating_inflight=2000, storage_media_type=codec.PROTOBUF, watch_window=200_000,
                 kubelet_port_resolver=None, audit=None, encryption_config=None,
                 service_cluster_ip_range="10.0.0.0/24", service_node_port_range=(30000, 32767),
                 tls_cert_file=None, tls_private_key_file=None, client_ca_file=None, service_account_key_files=(),
                 service_account_lookup=True, enable_bootstrap_token_auth=False, authentication_token_webhook=None,
                 anonymous_auth=True, authorization_policy_file=None, authorization_webhook_url=None, oidc=None,
                 component_endpoints=None, event_ttl=3600.0, kubelet_https=False, kubelet_certificate_authority=None,
                 kubelet_client_certificate=None, kubelet_client_key=None, basic_auth_file=None, requestheader=None,
                 authentication_token_webhook_config_file=None, authentication_token_webhook_cache_ttl=120.0,
                 authorization_webhook_config_file=None, authorization_webhook_cache_authorized_ttl=300.0,
                 authorization_webhook_cache_unauthorized_ttl=30.0, authorization_rbac_super_user=None,
                 cors_allowed_origins=(), request_timeout=None, min_request_timeout=1800.0, enable_logs_handler=True,
                 enable_swagger_ui=False, log_dir="/var/log", runtime_config=None, allow_privileged=True,
                 kubelet_preferred_address_types=("InternalIP", "ExternalIP", "Hostname", "InternalDNS", "ExternalDNS"),
                 kubelet_port=10250, kubelet_timeout=5.0, advertise_address=None, apiserver_count=1,
                 endpoint_reconciler_type="master-count", kubernetes_service_node_port=0, proxy_client_cert=None,
                 watch_cache_sizes=None, compaction_interval=0.0, delete_collection_workers=1):
        self.proxy_client_cert = proxy_client_cert          # (cert file, key file) for aggregated API servers
        # --watch-cache-sizes / --target-ram-mb: per-resource watch windows (plural -> events)
        self.watch_cache_sizes = dict(watch_cache_sizes or {})
        # --etcd-compaction-interval (`storage/etcd3/compact.go`): every interval the store's
        # history is compacted to the revision seen one interval earlier; 0 = never
        self.compaction_interval = float(compaction_interval or 0)
        self._compactor = None
        self.compactions = 0
        # --delete-collection-workers: concurrent deletes of one DELETE-collection call
        self.delete_collection_workers = max(1, int(delete_collection_workers))
        self.abac_policy_file = authorization_policy_file
        # --runtime-config: group/versions (and extensions/v1beta1 resources) switched off; every
        # served version is on by default here (the reference leaves alpha versions off)
        self.disabled_gv, self.disabled_res = parse_runtime_config(runtime_config)
        # --allow-privileged=false: privileged containers fail validation ("disallowed by cluster policy")
        self.allow_privileged = allow_privileged
        self.kubelet_address_types = tuple(kubelet_preferred_address_types)
        self.kubelet_port, self.kubelet_timeout = kubelet_port, kubelet_timeout
        # master endpoints (`pkg/master/controller.go`, reconcilers.go): --advertise-address,
        # --apiserver-count (master-count keeps that many addresses), none = not reconciled
        self.advertise_address = advertise_address
        self.apiserver_count = max(1, int(apiserver_count))
        if endpoint_reconciler_type not in ("master-count", "lease", "none"):
            raise ValueError(f"unknown endpoint reconciler {endpoint_reconciler_type!r}")
        self.endpoint_reconciler = endpoint_reconciler_type
        self.kubernetes_service_node_port = kubernetes_service_node_port
        # --cors-allowed-origins (regular expressions), --request-timeout (non-long-running requests
        # answer 504 after it; None = off), --min-request-timeout (watches without timeoutSeconds
        # end after a random time in [t, 2t)), --enable-logs-handler, --enable-swagger-ui
        import re as _re
        self.cors = [_re.compile(o) for o in cors_allowed_origins or ()]
        self.request_timeout = request_timeout
        self.min_request_timeout = min_request_timeout
        self.enable_logs_handler, self.enable_swagger_ui, self.log_dir = enable_logs_handler, enable_swagger_ui, log_dir
        self.requestheader = requestheader or None
        self.rbac_super_user = authorization_rbac_super_user
        self.authz_webhook = None
        if authorization_webhook_config_file:
            from ..client import clientcmd
            r = clientcmd.resolve_webhook(authorization_webhook_config_file)
            self.authz_webhook = (r.server, r.ssl_context, authorization_webhook_cache_authorized_ttl,
                                  authorization_webhook_cache_unauthorized_ttl)
        # kubelet connections (--kubelet-https, --kubelet-certificate-authority,
        # --kubelet-client-certificate/key; `pkg/kubelet/client` MakeTransport): without a CA the
        # kubelet's serving certificate is not verified, as in the reference
        self.kubelet_ssl = None
        if kubelet_https:
            from ..utils.tlsutil import client_context
            self.kubelet_ssl = client_context(kubelet_certificate_authority, kubelet_client_certificate, kubelet_client_key)
        self.kubelet_scheme = "https" if kubelet_https else "http"
        # --event-ttl: events expire this long after their last write (the reference stores them
        # with an etcd lease, `pkg/registry/core/event/storage/storage.go` ttlFunc)
        self.event_ttl = event_ttl
        self._reaper = None
        self.authorization_webhook_url = authorization_webhook_url
        self.authorization_modes = tuple(authorization_modes)
        self.tls = (tls_cert_file, tls_private_key_file, client_ca_file)
        from .service_alloc import ServiceAllocator
        from .extensions import Aggregator, CRDManager, WebhookDispatcher
        self.svc_alloc = ServiceAllocator(service_cluster_ip_range, service_node_port_range)
        self.webhooks = WebhookDispatcher(self)
        self.crds = CRDManager(self)
        self.aggregator = Aggregator(self)
        self.component_endpoints = component_endpoints if component_endpoints is not None else {
            "scheduler": "http://127.0.0.1:10251/healthz", "controller-manager": "http://127.0.0.1:10252/healthz"}
        from .openapi import OpenAPICache
        self.openapi = OpenAPICache(VERSION["gitVersion"])
        # encryption at rest (--experimental-encryption-provider-config): plural -> PrefixTransformers
        self.transformers = {}
        if encryption_config:
            from ..storage.value import load_encryption_config
            self.transformers = (encryption_config if isinstance(encryption_config, dict)
                                 and "kind" not in encryption_config else load_encryption_config(encryption_config))
        if store is None and os.environ.get("KAMD_APISERVER_DEFAULT_STORE"):
            # test plumbing: run an unchanged suite against another backend (an etcd v3 endpoint:
            # each API server under a key namespace of its own)
            from ..storage.etcd3_client import is_etcd3_address
            store = os.environ["KAMD_APISERVER_DEFAULT_STORE"]
            if is_etcd3_address(store):
                store += "#/kamd-" + secrets.token_hex(6)
        self.remote_address = store if isinstance(store, str) else None
        self.etcd_tls = etcd_tls      # (cafile, certfile, keyfile) for an https etcd endpoint
        self.rstore = None            # RemoteStore / Etcd3Store once started (shared mode)
        self.fanout = None            # FanoutClient: watches served by kamd-etcd (shared mode)
        from ..storage.etcd3_client import is_etcd3_address
        # the socket hand-off fan-out is a kamd-etcd feature; an etcd endpoint serves plain watches
        self.fanout_enabled = os.environ.get("KAMD_WATCH_FANOUT", "1") != "0" and \
            not is_etcd3_address(self.remote_address)
        # `store or ...` would be wrong: an empty store has len() == 0 and is falsy
        self.store = None if self.remote_address else (store if store is not None else MVCCStore())
        self._applied_rev = 0
        self.uncached: frozenset = frozenset()   # shared mode: resources read from the store
        self._rev_waiters: list = []  # heap of (rev, seq, future)
        self._waiter_seq = 0
        self._mine: dict = {}         # (key, rev) -> Entry committed by this worker
        self._rv_token = ("@rv-" + secrets.token_hex(12) + "@").encode()
        self._key_locks: dict = {}
        self.store_healthy = True
        self.caches: dict[str, ResourceCache] = {}
        self.strategies = {}
        self.storage_codec = codec.StorageCodec(storage_media_type)
        self.watch_window = watch_window
        self._store_res = {}          # etcd key segment (`pods`, `roles.rbac.authorization.k8s.io`) -> plural
        for ri in m.RESOURCES:
            self._install(ri)
        names = adm.DEFAULT_PLUGINS if admission_plugins is None else admission_plugins
        self.admission = adm.new_chain(names, self, admission_config)
        self.initializers_enabled = "Initializers" in names
        # admission webhooks are called only when their plugins are on the admission list
        self.mutating_webhooks_enabled = "MutatingAdmissionWebhook" in names
        self.validating_webhooks_enabled = "ValidatingAdmissionWebhook" in names
        self.authn = None
        if token_file or tokens or client_ca_file or service_account_key_files or enable_bootstrap_token_auth \
                or authentication_token_webhook or not anonymous_auth or oidc or basic_auth_file or requestheader \
                or authentication_token_webhook_config_file:
            from . import authn as an
            from ..native import crypto as _crypto
            toks = [TokenAuthenticator(token_file, tokens)] if (token_file or tokens) else []
            if enable_bootstrap_token_auth:
                toks.append(an.BootstrapTokenAuthenticator(self))
            if service_account_key_files:
                keys = []
                for f in service_account_key_files:
                    with open(f) as fh:
                        keys.append(_crypto.public_key(fh.read()))
                toks.append(an.ServiceAccountAuthenticator(keys, self, service_account_lookup))
            if authentication_token_webhook:
                toks.append(an.WebhookTokenAuthenticator(authentication_token_webhook, authentication_token_webhook_cache_ttl))
            if authentication_token_webhook_config_file:
                from ..client import clientcmd
                r = clientcmd.resolve_webhook(authentication_token_webhook_config_file)
                toks.append(an.WebhookTokenAuthenticator(r.server, authentication_token_webhook_cache_ttl, r.ssl_context))
            if oidc:
                toks.append(oidc if isinstance(oidc, an.OIDCAuthenticator) else an.OIDCAuthenticator(**oidc))
            # request authenticators in the reference's order: front proxy, x509, basic auth
            reqs = []
            if requestheader:
                with open(requestheader["client_ca_file"]) as f:
                    rh_ca = f.read()
                reqs.append(an.RequestHeaderAuthenticator(
                    rh_ca, requestheader.get("allowed_names") or (),
                    requestheader.get("username_headers") or ("X-Remote-User",),
                    requestheader.get("group_headers") or ("X-Remote-Group",),
                    requestheader.get("extra_headers_prefix") or ("X-Remote-Extra-",)))
            if client_ca_file:
                ca_pem = None
                if requestheader:       # the listener trusts both CAs: bind x509 users to the client CA
                    with open(client_ca_file) as f:
                        ca_pem = f.read()
                reqs.append(an.X509Authenticator(ca_pem))
            if basic_auth_file:
                reqs.append(an.BasicAuthenticator(basic_auth_file))
            self.authn = an.UnionAuthenticator(reqs, toks, anonymous_auth)
        self.authz = build_authorizer(authorization_modes, self)
        self.max_inflight = max_requests_inflight
        self.max_mutating = max_mutating_inflight
        self.inflight = 0
        self.inflight_mut = 0
        self.http = HTTPServer(self._entry if self.cors else self.handle, request_timeout=self.request_timeout,
                               long_running=self._long_running, timeout_response=_TIMEOUT_RESPONSE)
        self.insecure_http = None
        self.insecure_port = None
        self.kubelet_port_resolver = kubelet_port_resolver
        self.audit = audit            # audit.AuditLogger or None
        self.enable_profiling = True  # --profiling (reference default true)
        # fork fix: node -> {(resource, deviceID): pod key}
        self.node_devices: dict[str, dict[tuple, str]] = {}
        self.metrics = Registry()
        self.m_requests = self.metrics.counter("apiserver_request_count", "Counter of apiserver requests",
                                               ("verb", "resource", "subresource", "code"))
        self.m_latency = self.metrics.histogram("apiserver_request_latencies_seconds", "Request latency",
                                                ("verb", "resource"), (0.0005, 0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 5))
        self.m_watchers = self.metrics.gauge("apiserver_registered_watchers", "Number of watchers", ("kind",))
        self.m_inflight = self.metrics.gauge("apiserver_current_inflight_requests", "In-flight requests", ("requestKind",))
        self.m_dropped = self.metrics.counter("apiserver_dropped_requests", "Requests dropped with 429", ("requestKind",))
        self.m_fanout = self.metrics.counter("apiserver_watch_fanout_handoffs_total",
                                             "Watches handed to the store's native fan-out", ("resource",))
        self.m_retries = self.metrics.counter("apiserver_shared_store_retries_total",
                                              "Requests re-run because this worker's cache lagged the shared store",
                                              ("reason",))
        self.metrics.register_collector(self._collect)
        if self.store is not None:
            self._load_from_store()
            _run_sync(self.bootstrap())

    @property
    def revision(self) -> int:
        """Latest revision reflected in this server's caches."""
        return self.store.revision if self.store is not None else self._applied_rev

    # ------------------------------------------------------------------
    def _install(self, ri):
        self.caches[ri.plural] = ResourceCache(ri.plural, self.watch_cache_sizes.get(ri.plural, self.watch_window))
        self.strategies[ri.plural] = strategy_for(ri)
        self._store_res[m.prefix_for(ri).split("/")[2]] = ri.plural

    def install_resource(self, ri):
        """Serve a new resource (CRD established)."""
        m.register(ri)
        if ri.plural not in self.caches:
            self._install(ri)

    def uninstall_resource(self, ri):
        self.caches.pop(ri.plural, None)
        self.strategies.pop(ri.plural, None)
        self._store_res = {k: v for k, v in self._store_res.items() if v != ri.plural}
        m.unregister(ri)

    def _observe(self, plural, obj, deleted):
        """Side effects of objects entering / leaving the caches on every worker."""
        if plural == "customresourcedefinitions" and obj is not None:
            self.crds.observe(obj, deleted)

    def _cache_for_key(self, key):
        parts = key.split("/", 3)
        if len(parts) <= 3:
            return None, None
        plural = self._store_res.get(parts[2])
        return plural, (self.caches.get(plural) if plural else None)

    def _seal(self, plural, key, data: bytes) -> bytes:
        t = self.transformers.get(plural)
        return data if t is None else t.to_storage(data, key.encode())

    def _unseal(self, key, data: bytes) -> bytes:
        if data[:8] != ENC_PREFIX:
            return data
        plural, _ = self._cache_for_key(key)
        t = self.transformers.get(plural)
        if t is None:
            raise APIError(500, "InternalError", f"stored value of {key} is encrypted but no provider is configured")
        return t.from_storage(data, key.encode())[0]

    def _collect(self):
        out = ["# TYPE etcd_object_counts gauge"]
        for plural, c in sorted(self.caches.items()):
            if c.by_key:
                out.append(f'etcd_object_counts{{resource="{plural}"}} {len(c.by_key)}')
        out.append("# TYPE apiserver_storage_revision gauge")
        out.append(f"apiserver_storage_revision {self.revision}")
        return out

    def _load_from_store(self):
        """Rebuild the watch caches after a restart (WAL replay)."""
        if not self.store.revision or self.store.revision <= 1:
            return
        for ri in m.RESOURCES:
            kvs, _, _ = self.store.range(m.prefix_for(ri))
            cache = self.caches[ri.plural]
            for kv in kvs:
                obj = self.storage_codec.decode(self._unseal(kv.key, kv.value))
                obj.setdefault("metadata", {})["resourceVersion"] = str(kv.mod_rev)
                raw = codec.dumpb(obj)
                cache.by_key[kv.key] = cache.make_entry(obj, raw, kv.mod_rev)
                if ri.plural == "pods":
                    self._index_pod(kv.key, None, obj)
                self._observe(ri.plural, obj, False)
            cache.rev = self.store.revision

    async def bootstrap(self):
        for ns in ("default", "kube-system", "kube-public"):
            if self.get_object("namespaces", None, ns) is None:
                try:
                    await self._retrying(lambda: self.create(m.BY_PLURAL["namespaces"], None,
                                                             {"metadata": {"name": ns}}, admit=False))
                except APIError as e:
                    if e.code != 409:   # another worker created it first
                        raise
        if "RBAC" in self.authorization_modes:
            from .bootstrappolicy import ensure_bootstrap_policy
            await ensure_bootstrap_policy(self)
        # the `kubernetes` service on the first IP of the service range
        # (pkg/master/controller.go CreateOrUpdateMasterServiceIfNeeded)
        if self.get_object("services", "default", "kubernetes") is None:
            svc = {"metadata": {"name": "kubernetes", "namespace": "default",
                                "labels": {"component": "apiserver", "provider": "kubernetes"}},
                   "spec": {"clusterIP": self.svc_alloc.kubernetes_ip, "type": "ClusterIP", "sessionAffinity": "None",
                            "ports": [{"name": "https", "port": 443, "protocol": "TCP", "targetPort": 6443}]}}
            if self.kubernetes_service_node_port:     # --kubernetes-service-node-port
                svc["spec"]["type"] = "NodePort"
                svc["spec"]["ports"][0]["nodePort"] = self.kubernetes_service_node_port
            try:
                await self._retrying(lambda: self.create(m.BY_PLURAL["services"], "default", svc, admit=False))
            except APIError as e:
                if e.code not in (409, 422):
                    raise

    # ------------------------------------------------------------------
    # shared-store mode
    async def _start_remote(self):
        from ..storage.etcd3_client import connect_store
        self.rstore = await connect_store(self.remote_address, self.etcd_tls)
        from ..storage.remote import FanoutClient
        self.fanout = FanoutClient.for_store(self.remote_address) if self.fanout_enabled else None
        self.uncached = self._uncached_resources()
        excl = tuple(m.prefix_for(m.BY_PLURAL[p]) for p in sorted(self.uncached))
        # one RANGE is an atomic snapshot (the store is single-threaded); watch from its revision
        kvs, _, rev = await self.rstore.range("/registry/")
        for kv in kvs:
            if not (excl and kv.key.startswith(excl)):
                self._ingest(0, kv, dispatch=False)
        self._applied_rev = rev
        for c in self.caches.values():
            c.rev = rev
        await self.rstore.watch("/registry/", rev, self._on_store_event, exclude=excl)
        await self.bootstrap()

    def _uncached_resources(self):
        """Resources this shared-mode worker serves from the store instead of a watch cache:
        pods and events, unless something here must read them synchronously (the Node
        authorizer's pod graph) or their watches cannot be handed to the store's fan-out
        (encrypted storage, TLS client connections). KAMD_SHARED_CACHE_ALL=1 keeps
        every resource cached."""
        if os.environ.get("KAMD_SHARED_CACHE_ALL") == "1" or self.fanout is None or self.tls[0] \
                or "Node" in self.authorization_modes:
            return frozenset()
        return frozenset(p for p in ("pods", "events") if p not in self.transformers)

    def _storage_encode(self, ri, obj):
        """The storage bytes of obj; a field outside the reference schema is a 422, never a silent
        drop (the protobuf encoder refuses what it cannot represent)."""
        try:
            return self.storage_codec.encode(obj)
        except pb.ProtobufError as e:
            from ..api.validation import FieldError
            raise invalid(ri, m.name_of(obj), [FieldError("Invalid value", e.path or "<object>", str(e).split(": ", 1)[-1])])

    def _entry_from_kv(self, plural, kv):
        """Entry for a stored value without decoding the object: shared-store values carry the
        index header (fields, labels) in front of the object JSON."""
        v = kv.value
        if v[:3] == _FRAME:
            hl = int.from_bytes(v[3:7], "little")
            fields, labels = codec.loads(v[7:7 + hl])
            body = v[7 + hl:]
            if body[:4] == codec.MAGIC:
                # protobuf storage: the JSON for GET/LIST/watch payloads (resourceVersion from the
                # key's mod revision — etcd3 never stores it) is made on first use; protobuf
                # clients get the envelope itself
                return Entry(None, None, kv.mod_rev, fields, labels, body)
            return Entry(None, body, kv.mod_rev, fields, labels)
        obj, raw = self._decode_value(kv)
        return self.caches[plural].make_entry(obj, raw, kv.mod_rev)

    async def _store_entries(self, ri, ns=None, label_sel=None, field_sel=None):
        """(entries, revision) of an uncached resource straight from the store, key order."""
        kvs, _, rev = await self.rstore.range(m.prefix_for(ri, ns if ri.namespaced else None))
        out = []
        for kv in kvs:
            e = self._entry_from_kv(ri.plural, kv)
            if label_sel is not None and not label_sel.matches(e.labels):
                continue
            if field_sel is not None and not field_sel.matches(e.fields):
                continue
            out.append(e)
        return out, rev

    def _decode_value(self, kv):
        v = kv.value
        if v[:3] == _FRAME:
            v = v[7 + int.from_bytes(v[3:7], "little"):]
        if v[:8] == ENC_PREFIX:
            obj = self.storage_codec.decode(self._unseal(kv.key, v))
            obj.setdefault("metadata", {})["resourceVersion"] = str(kv.mod_rev)
            return obj, codec.dumpb(obj)
        if v[:4] == codec.MAGIC:
            obj = self.storage_codec.decode(v)
            obj.setdefault("metadata", {})["resourceVersion"] = str(kv.mod_rev)
            return obj, codec.dumpb(obj)
        return codec.loads(v), v

    def _ingest(self, t, kv, dispatch=True):
        _, cache = self._cache_for_key(kv.key)
        if cache is None:
            return
        entry = self._mine.pop((kv.key, kv.mod_rev), None)
        if entry is None:
            # another worker's write: keep the bytes, decode only the small index header; the
            # object itself is decoded on first use (Entry.obj)
            entry = self._entry_from_kv(cache.resource, kv)
        prev = cache.by_key.get(kv.key)
        plural = cache.resource
        if not dispatch:
            cache.by_key[kv.key] = entry
            if plural == "customresourcedefinitions":
                self._observe(plural, entry.obj, False)
            return
        etype = DELETED if t == wire.OP_DELETE else (MODIFIED if prev is not None else ADDED)
        if etype == DELETED and prev is None:
            return
        cache.apply(etype, kv.key, entry, prev)
        if plural == "customresourcedefinitions":
            self._observe(plural, entry.obj if etype != DELETED else prev.obj, etype == DELETED)

    def _on_store_event(self, t, kv):
        if t == wire.PROGRESS:        # only excluded (uncached) keys changed, up to revision `kv`
            self._advance(kv)
            return
        if t is None:
            if self.store_healthy:
                log.error("store watch stream ended; this API server worker is now unhealthy")
            self.store_healthy = False
            for _, _, f in self._rev_waiters:
                if not f.done():
                    f.set_exception(APIError(503, "ServiceUnavailable", "storage unavailable"))
            self._rev_waiters.clear()
            return
        try:
            self._ingest(t, kv)
        except Exception:
            log.exception("failed to apply store event %s@%d", kv.key, kv.mod_rev)
        self._advance(kv.mod_rev)

    def _advance(self, rev):
        if rev > self._applied_rev:
            self._applied_rev = rev
            w = self._rev_waiters
            if w and w[0][0] <= rev:
                import heapq
                while w and w[0][0] <= rev:
                    _, _, f = heapq.heappop(w)
                    if not f.done():
                        f.set_result(None)

    async def _wait_applied(self, rev, timeout=30.0):
        if rev <= self._applied_rev:
            return
        if not self.store_healthy:
            raise APIError(503, "ServiceUnavailable", "storage unavailable")
        import heapq
        f = asyncio.get_running_loop().create_future()
        self._waiter_seq += 1
        heapq.heappush(self._rev_waiters, (rev, self._waiter_seq, f))
        try:
            await asyncio.wait_for(f, timeout)
        except asyncio.TimeoutError:
            raise APIError(504, "Timeout", f"timed out waiting for revision {rev} to be observed")

    async def _retrying(self, op, attempts=64):
        """Re-run an operation whose compare failed on a stale cache, or which missed an object
        this worker has not seen yet (shared mode)."""
        for i in range(attempts):
            try:
                return await op()
            except _Stale as e:
                self.m_retries.labels("stale").inc()
                if i == attempts - 1:
                    raise APIError(409, "Conflict", "the object has been modified concurrently; please retry")
                await self._wait_applied(e.rev)
            except _Missing as e:
                self.m_retries.labels("miss").inc()
                kv = await self.rstore.get(e.key)
                if kv is None or i == attempts - 1:
                    raise e.error
                await self._wait_applied(kv.mod_rev)

    async def _async_existing(self, ri, namespace, name):
        return await self._aexisting(ri, namespace, name)

    async def _aexisting(self, ri, namespace, name):
        """(key, Entry) of an existing object: from the store for uncached resources, else from
        this worker's cache (`_existing`)."""
        if ri.plural in self.uncached:
            key = m.key_for(ri, namespace, name)
            kv = await self.rstore.get(key)
            if kv is None:
                raise not_found(ri, name)
            return key, self._entry_from_kv(ri.plural, kv)
        if self.rstore is None:
            return self._existing(ri, namespace, name)
        # shared store: a cache miss may only mean this worker lags the store
        return await self._retrying(lambda: asyncio.sleep(0, self._existing(ri, namespace, name)), attempts=4)

    def _claim_keys(self, ri, obj):
        """Keys that must be absent in the store for `obj` to be written (shared mode): GPU device
        assignments of pods, ClusterIPs / NodePorts of services."""
        if ri.plural == "pods":
            return self._device_keys(obj)
        if ri.plural == "services":
            return self.svc_alloc.claim_keys(obj)
        return set()

    @staticmethod
    def _device_keys(pod):
        if pod is None or core.pod_is_terminal(pod):
            return set()
        node = (pod.get("spec") or {}).get("nodeName")
        if not node:
            return set()
        return {f"{DEVICE_PREFIX}{node}/{rn}/{i}" for rn, ids in core.pod_assigned_devices(pod).items() for i in ids}

    async def _commit_remote(self, ri, key, etype, obj, prev):
        md = obj["metadata"]
        tok = self._rv_token
        cache = self.caches[ri.plural]
        sealed = ri.plural in self.transformers
        json_storage = self.storage_codec.media_type == codec.JSON and not sealed
        if not json_storage and not sealed and self.storage_codec.media_type == codec.PROTOBUF:
            # kinds outside the protobuf schema (custom resources) are stored as JSON
            json_storage = pb.message_of(obj) is None
        # value framing: [00 'K' 'H' | u32 len | index header (fields, labels) | object]
        hdr = codec.dumpb([cache.index_fields(obj), md.get("labels") or {}])
        frame = _FRAME + len(hdr).to_bytes(4, "little") + hdr
        if json_storage:
            md["resourceVersion"] = tok.decode()
            raw_t = codec.dumpb(obj)
            stored = frame + raw_t
        else:
            md.pop("resourceVersion", None)
            raw_t = None
            enc = self._storage_encode(ri, obj)
            # unsealed protobuf keeps the index frame: the store's fan-out filters on it and
            # transcodes the object for JSON watchers
            stored = self._seal(ri.plural, key, enc) if sealed else frame + enc
        cmps = [(wire.CMP_MOD_REV, key, prev.rev if prev is not None else 0, None)]
        if etype == DELETED and sealed:
            # no plaintext index header or tombstone for encrypted resources
            ops = [(wire.OP_DELETE_TOMBSTONE, key, self._seal(ri.plural, key, codec.dumpb(obj)), tok)]
        elif etype == DELETED:
            tomb = raw_t if raw_t is not None else stored[len(frame):]
            ops = [(wire.OP_DELETE_TOMBSTONE, key, frame + tomb, tok)]
        elif json_storage:
            ops = [(wire.OP_PUT_INJECT, key, stored, tok)]
        else:
            ops = [(wire.OP_PUT, key, stored)]   # binary values are never rewritten
        if ri.plural in ("pods", "services"):
            old_d = self._claim_keys(ri, prev.obj if prev is not None else None)
            new_d = set() if etype == DELETED else self._claim_keys(ri, obj)
            kb = key.encode()
            for dk in sorted(new_d - old_d):
                cmps.append((wire.CMP_ABSENT, dk, 0, None))
                ops.append((wire.OP_PUT, dk, kb))
            for dk in sorted(old_d - new_d):
                ops.append((wire.OP_DELETE, dk, None))
        cache = self.caches[ri.plural]
        uncached = ri.plural in self.uncached
        done = []

        def on_ok(rev):
            rs = str(rev)
            md["resourceVersion"] = rs
            pbv = None
            if raw_t is not None:
                raw = raw_t.replace(tok, rs.encode())
            elif not sealed and etype != DELETED:
                # what every other worker (and the store's fan-out) serves for this revision: the
                # stored envelope (protobuf clients) or its JSON form (Go omitempty: no empty maps
                # / lists), made only if a JSON client asks (Entry.raw)
                raw, pbv = None, stored[len(frame):]
            else:
                raw = codec.dumpb(obj)
            entry = cache.make_entry(obj, raw, rev)
            entry.pbv = pbv
            if not uncached:
                self._mine[(key, rev)] = entry
            done.append(entry)

        res = await self.rstore.txn(cmps, ops, on_ok)
        if not res.ok:
            if res.failed == 0:
                if uncached:
                    # read from the store, not a lagging cache: the object really changed
                    if etype == ADDED:
                        raise already_exists(ri, m.name_of(obj))
                    raise _Stale(0)
                raise _Stale(res.rev)
            owner = res.current.value.decode() if res.current is not None else "?"
            claim = cmps[res.failed][1]
            if not claim.startswith(DEVICE_PREFIX):
                raise APIError(409, "Conflict", f"{claim.rsplit('/', 1)[-1]} is already allocated to {owner}")
            dev = claim[len(DEVICE_PREFIX):]
            raise APIError(409, "Conflict", f"device {dev} is already assigned to {owner.rsplit('/', 2)[-2]}/{owner.rsplit('/', 1)[-1]}")
        if uncached:
            return done[0]
        await self._wait_applied(res.rev)
        self._mine.pop((key, res.rev), None)
        return done[0]

    # ------------------------------------------------------------------
    # object-level API (admission plugins, controllers in-process, tests)
    def get_object(self, plural, namespace, name):
        if plural in self.uncached:
            raise RuntimeError(f"{plural} are not cached by this shared-store worker; read them from the store")
        ri = m.BY_PLURAL[plural]
        e = self.caches[plural].get(m.key_for(ri, namespace, name))
        return e.obj if e else None

    def list_objects(self, plural, namespace=None):
        if plural in self.uncached:
            raise RuntimeError(f"{plural} are not cached by this shared-store worker; read them from the store")
        ri = m.BY_PLURAL[plural]
        prefix = m.prefix_for(ri, namespace if ri.namespaced else None)
        return [e.obj for k, e in self.caches[plural].by_key.items() if k.startswith(prefix)]

    # ------------------------------------------------------------------
    # commit path
    async def _commit(self, ri, key, etype, obj, prev):
        """Write obj (already fully prepared) to the store and the cache. Returns Entry."""
        if self.rstore is not None:
            return await self._commit_remote(ri, key, etype, obj, prev)
        return self._commit_local(ri, key, etype, obj, prev)

    def _commit_local(self, ri, key, etype, obj, prev):
        rev = self.store.revision + 1
        obj["metadata"]["resourceVersion"] = str(rev)
        raw = codec.dumpb(obj)
        stored = raw if self.storage_codec.media_type == codec.JSON else self._storage_encode(ri, obj)
        if ri.plural in self.transformers:
            stored = self._seal(ri.plural, key, stored)
        if etype == ADDED:
            ev = self.store.create(key, stored)
            if ev is None:
                raise already_exists(ri, m.name_of(obj))
        elif etype == MODIFIED:
            ok, ev = self.store.update(key, stored, prev.rev)
            if not ok:
                raise conflict(ri, m.name_of(obj), "the object has been modified; please apply your changes to the latest version and try again")
        else:
            ok, ev = self.store.delete(key, prev.rev)
            if not ok:
                raise conflict(ri, m.name_of(obj), "the object has been modified")
        assert ev.kv.mod_rev == rev, (ev.kv.mod_rev, rev)
        cache = self.caches[ri.plural]
        entry = cache.make_entry(obj, raw, rev)
        if ri.plural == "pods":
            self._index_pod(key, prev.obj if prev else None, None if etype == DELETED else obj)
        cache.apply(etype, key, entry, prev)
        if ri.plural == "customresourcedefinitions":
            self._observe(ri.plural, obj, etype == DELETED)
        return entry

    def _index_pod(self, key, old, new):
        if old is not None:
            node = (old.get("spec") or {}).get("nodeName")
            if node:
                idx = self.node_devices.get(node)
                if idx:
                    for rn, ids in core.pod_assigned_devices(old).items():
                        for i in ids:
                            if idx.get((rn, i)) == key:
                                del idx[(rn, i)]
        if new is not None and not core.pod_is_terminal(new):
            node = (new.get("spec") or {}).get("nodeName")
            if node:
                idx = self.node_devices.setdefault(node, {})
                for rn, ids in core.pod_assigned_devices(new).items():
                    for i in ids:
                        idx[(rn, i)] = key

    # ------------------------------------------------------------------
    # verbs
    async def create(self, ri, namespace, obj, user=None, admit=True, subresource=""):
        if not isinstance(obj, dict):
            raise bad_request("body must be a JSON object")
        init_object_meta(obj, ri, namespace)
        defaults.apply(ri.kind, obj)       # the scheme's SetDefaults_* before validation
        strat = self.strategies[ri.plural]
        strat.prepare_create(obj)
        if ri.plural == "certificatesigningrequests":
            # the requester's identity is recorded by the server, never trusted from the body
            sp = obj.setdefault("spec", {})
            u = user or ANONYMOUS
            sp["username"], sp["uid"], sp["groups"] = u.name, u.uid or "", list(u.groups or ())
            obj["status"] = {}
        ns = m.namespace_of(obj) if ri.namespaced else None
        if admit:
            a = adm.Attributes(adm.CREATE, ri.plural, subresource, ns, m.name_of(obj), obj, None, user, ri.kind)
            if self.admission._prepare:
                try:
                    await self.admission.prepare(a)
                except adm.AdmissionError as e:
                    raise APIError(e.code, e.reason, str(e))
            self._admit(a)
            obj = await self._mutating_webhooks(a, ri)
        if ri.plural == "services":
            return await self._create_service(ri, ns, obj, a if admit else None)
        errs = self._validate_new(ri, strat, obj)
        if errs:
            raise invalid(ri, m.name_of(obj), errs)
        key = m.key_for(ri, ns, m.name_of(obj))
        if admit:
            self._validate_admission(a)
            await self._validating_webhooks(a, ri)
            if key in self.caches[ri.plural].by_key:
                raise already_exists(ri, m.name_of(obj))
            await self._charge_admission(a)
        if key in self.caches[ri.plural].by_key:
            raise already_exists(ri, m.name_of(obj))
        return await self._commit(ri, key, ADDED, obj, None)

    # ------------------------------------------------------------------ extension hooks
    _NO_WEBHOOKS = ("mutatingwebhookconfigurations", "validatingwebhookconfigurations")

    async def _mutating_webhooks(self, a, ri):
        if self.mutating_webhooks_enabled and ri.plural not in self._NO_WEBHOOKS and self.webhooks.has_any():
            await self.webhooks.run(a, ri, True)
        return a.obj

    async def _validating_webhooks(self, a, ri):
        if self.validating_webhooks_enabled and ri.plural not in self._NO_WEBHOOKS and self.webhooks.has_any():
            await self.webhooks.run(a, ri, False)

    def _validate_new(self, ri, strat, obj, old=None):
        if not self.allow_privileged and ri.plural == "pods":
            from ..api.validation import FieldError
            spec = obj.get("spec") or {}
            bad = [FieldError("Forbidden", f"spec.{key}[{i}].securityContext.privileged", "disallowed by cluster policy")
                   for key in ("initContainers", "containers") for i, c in enumerate(spec.get(key) or ())
                   if (c.get("securityContext") or {}).get("privileged")]
            if bad:
                return bad + list(strat.validate(obj) if old is None else strat.validate_update(obj, old))
        if ri.plural == "customresourcedefinitions":
            from .extensions import validate_crd
            errs = validate_crd(obj)
            if not errs and old is None:
                self.crds.prepare(obj)
            return errs
        errs = strat.validate(obj) if old is None else strat.validate_update(obj, old)
        if ri.plural in self.crds.schemas:
            from ..api.validation import FieldError
            for e in self.crds.validate_object(ri, obj):
                fld, _, rest = e.partition(": ")
                typ, _, detail = rest.partition(": ")
                errs = list(errs) + [FieldError(typ, fld, detail)]
        return errs

    async def _create_service(self, ri, ns, obj, a):
        from .service_alloc import AllocationError
        strat = self.strategies[ri.plural]
        key = m.key_for(ri, ns, m.name_of(obj))
        base = fast_copy(obj)
        for attempt in range(8):
            obj = fast_copy(base)
            try:
                auto = self.svc_alloc.allocate(obj, self.list_objects("services"))
            except AllocationError as e:
                raise APIError(e.code, "Invalid" if e.code == 422 else "InternalError", str(e))
            errs = strat.validate(obj)
            if errs:
                raise invalid(ri, m.name_of(obj), errs)
            if key in self.caches[ri.plural].by_key:
                raise already_exists(ri, m.name_of(obj))
            if a is not None:
                a.obj = obj
                self._validate_admission(a)
                if attempt == 0:
                    await self._charge_admission(a)
            try:
                return await self._commit(ri, key, ADDED, obj, None)
            except APIError as e:
                # another API server worker allocated the same IP / port first: pick again
                if e.code != 409 or "already allocated" not in e.message or not auto or attempt == 7:
                    raise

    def _admit(self, a):
        try:
            self.admission.admit(a)
        except adm.AdmissionError as e:
            raise APIError(e.code, e.reason, str(e))

    def _validate_admission(self, a):
        try:
            self.admission.validate(a)
        except adm.AdmissionError as e:
            raise APIError(e.code, e.reason, str(e))

    async def _charge_admission(self, a):
        try:
            await self.admission.charge(a)
        except adm.AdmissionError as e:
            raise APIError(e.code, e.reason, str(e))

    async def quota_objects(self, namespace, fresh=False):
        """The namespace's ResourceQuotas for quota admission; `fresh` re-reads them from the
        store (a shared-store worker's cache may lag a quota another worker just charged)."""
        if fresh and self.rstore is not None:
            return [e.obj for e in (await self._store_entries(m.BY_PLURAL["resourcequotas"], namespace))[0]]
        return self.list_objects("resourcequotas", namespace)

    async def write_quota_status(self, q):
        """Persist admission's charged status.used with the quota's resourceVersion (409 when
        another request charged it first)."""
        await self.update(m.BY_PLURAL["resourcequotas"], m.namespace_of(q), m.name_of(q), q, None, "status")

    def _existing(self, ri, namespace, name):
        key = m.key_for(ri, namespace, name)
        e = self.caches[ri.plural].get(key)
        if e is None:
            if self.rstore is not None:
                raise _Missing(key, not_found(ri, name))
            raise not_found(ri, name)
        return key, e

    async def update(self, ri, namespace, name, obj, user=None, subresource=""):
        if not isinstance(obj, dict):
            raise bad_request("body must be a JSON object")
        key, prev = await self._aexisting(ri, namespace, name)
        old = prev.obj
        obj = dict(obj)
        om = old["metadata"]
        nm = obj["metadata"] = dict(obj.get("metadata") or {})
        if nm.get("name") and nm["name"] != name:
            raise bad_request("the name of the object does not match the name on the URL")
        want_rv = nm.get("resourceVersion")
        if want_rv and want_rv != om.get("resourceVersion"):
            raise conflict(ri, name, "the object has been modified; please apply your changes to the latest version and try again")
        if nm.get("uid") and nm["uid"] != om.get("uid"):
            raise conflict(ri, name, "Precondition failed: UID in precondition does not match")
        for k in ("uid", "creationTimestamp", "name", "namespace", "selfLink", "generation", "deletionTimestamp",
                  "deletionGracePeriodSeconds"):
            if k in om:
                nm[k] = om[k]
            else:
                nm.pop(k, None)
        obj["kind"], obj["apiVersion"] = ri.kind, ri.group_version
        strat = self.strategies[ri.plural]
        if subresource == "approval" and ri.plural == "certificatesigningrequests":
            # CSR approval subresource: only status.conditions may change
            # (pkg/registry/certificates/certificates/strategy.go approvalStrategy)
            conds = (obj.get("status") or {}).get("conditions") or []
            obj = fast_copy(old)
            obj["metadata"] = nm
            obj.setdefault("status", {})["conditions"] = conds
        elif subresource == "status":
            strat.prepare_status_update(obj, old)
        elif subresource == "":
            defaults.apply(ri.kind, obj)
            strat.prepare_update(obj, old)
            if strat.bump_generation and "generation" in om:
                if {k: v for k, v in obj.items() if k not in ("metadata", "status")} != \
                        {k: v for k, v in old.items() if k not in ("metadata", "status")} or \
                        (strat.generation_on_annotations and (nm.get("annotations") or {}) != (om.get("annotations") or {})):
                    nm["generation"] = om["generation"] + 1
        a = adm.Attributes(adm.UPDATE, ri.plural, subresource, namespace, name, obj, old, user, ri.kind)
        self._admit(a)
        obj = await self._mutating_webhooks(a, ri)
        nm = obj["metadata"]
        # a status update keeps the (already validated) spec, so only metadata + status are checked
        # (reference: ValidatePodStatusUpdate / ValidateNodeUpdate on the status subresource)
        errs = self._validate_new(ri, strat, obj, old) if subresource == "" else strat.validate_status(obj)
        if errs:
            raise invalid(ri, name, errs)
        self._validate_admission(a)
        await self._validating_webhooks(a, ri)
        if subresource == "":
            await self._charge_admission(a)
        # finalizers drained on an object that is being deleted -> delete it now
        if nm.get("deletionTimestamp") and not nm.get("finalizers") and self._grace_expired(ri, obj):
            return await self._commit(ri, key, DELETED, obj, prev)
        nm["resourceVersion"] = om.get("resourceVersion")
        if obj == old:
            return prev  # no-op update: no write, no event (etcd3 GuaranteedUpdate byte-equal short cut)
        return await self._commit(ri, key, MODIFIED, obj, prev)

    def _grace_expired(self, ri, obj):
        if ri.plural != "pods":
            return True
        g = obj["metadata"].get("deletionGracePeriodSeconds")
        return not g

    async def guaranteed_update(self, ri, namespace, name, fn, user=None, subresource=""):
        """Internal read-modify-write (used by binding, eviction)."""
        key, prev = await self._aexisting(ri, namespace, name)
        obj = fast_copy(prev.obj)
        fn(obj)
        return await self._commit(ri, key, MODIFIED, obj, prev)

    async def patch(self, ri, namespace, name, content_type, patch_body, user=None, subresource=""):
        key, prev = await self._aexisting(ri, namespace, name)
        try:
            patch = codec.loads(patch_body)
            # merge / strategic patches build new dicts along the patched paths only and share
            # the rest with the cached object (copy-on-write); update() never mutates shared parts
            new = apply_patch(content_type, prev.obj, patch)
        except (JSONPatchError, ValueError) as e:
            if isinstance(e, ValueError) and "unsupported patch type" in str(e):
                raise APIError(415, "UnsupportedMediaType", str(e))
            raise APIError(422, "Invalid", f"the patch could not be applied: {e}")
        if not isinstance(patch, dict) or "resourceVersion" not in (patch.get("metadata") or {}):
            new.setdefault("metadata", {})["resourceVersion"] = prev.obj["metadata"].get("resourceVersion")
        return await self.update(ri, namespace, name, new, user, subresource)

    async def delete(self, ri, namespace, name, opts=None, user=None):
        """Returns (Entry, deleted_now)."""
        opts = opts or {}
        key, prev = await self._aexisting(ri, namespace, name)
        old = prev.obj
        pre = opts.get("preconditions") or {}
        if pre.get("uid") and pre["uid"] != old["metadata"].get("uid"):
            raise conflict(ri, name, f"Precondition failed: UID in precondition: {pre['uid']}, UID in object meta: {old['metadata'].get('uid')}")
        a = adm.Attributes(adm.DELETE, ri.plural, "", namespace, name, None, old, user, ri.kind, opts)
        self._admit(a)
        self._validate_admission(a)
        await self._validating_webhooks(a, ri)
        if ri.plural == "customresourcedefinitions" and m.name_of(old) in self.crds.installed:
            # finalizer controller: custom objects go before their definition
            cri = self.crds.installed[m.name_of(old)]
            for o in list(self.list_objects(cri.plural)):
                try:
                    await self.delete(cri, m.namespace_of(o) or None, m.name_of(o), {}, user)
                except APIError as e:
                    if e.code != 404:
                        raise
        strat = self.strategies[ri.plural]
        obj = dict(old)                      # copy-on-write: only metadata/status are rewritten
        om = obj["metadata"] = dict(old["metadata"])
        if "status" in old and isinstance(old["status"], dict):
            obj["status"] = dict(old["status"])
        grace = strat.graceful_seconds(old, opts)
        fins = list(om.get("finalizers") or [])
        pol = opts.get("propagationPolicy")
        if opts.get("orphanDependents") is True:
            pol = "Orphan"
        if pol == "Orphan" and "orphan" not in fins and ri.plural not in ("pods", "events"):
            fins.append("orphan")
        elif pol == "Foreground" and "foregroundDeletion" not in fins:
            fins.append("foregroundDeletion")
        if ri.plural == "namespaces":
            if (obj.get("spec") or {}).get("finalizers"):
                if not om.get("deletionTimestamp"):
                    om["deletionTimestamp"] = now_rfc3339()
                    obj.setdefault("status", {})["phase"] = "Terminating"
                    return (await self._commit(ri, key, MODIFIED, obj, prev)), False
                return prev, False
        if grace > 0:
            cur = om.get("deletionGracePeriodSeconds")
            if cur is not None and cur <= grace:
                return prev, False  # already deleting with a shorter grace period
            om["deletionTimestamp"] = deletion_stamp(grace)
            om["deletionGracePeriodSeconds"] = grace
            if fins:
                om["finalizers"] = fins
            return (await self._commit(ri, key, MODIFIED, obj, prev)), False
        if fins:
            changed = om.get("finalizers") != fins or not om.get("deletionTimestamp") or om.get("deletionGracePeriodSeconds")
            om["finalizers"] = fins
            om.setdefault("deletionTimestamp", now_rfc3339())
            om["deletionGracePeriodSeconds"] = 0
            if not changed:
                return prev, False
            return (await self._commit(ri, key, MODIFIED, obj, prev)), False
        om["deletionGracePeriodSeconds"] = 0
        om.setdefault("deletionTimestamp", now_rfc3339())
        return (await self._commit(ri, key, DELETED, obj, prev)), True

    async def bind(self, namespace, name, binding, user=None):
        """POST pods/{name}/binding (fork F6) with the duplicate-device guard."""
        ri = m.BY_PLURAL["pods"]
        key, prev = await self._aexisting(ri, namespace, name)
        a = adm.Attributes(adm.CREATE, "pods", "binding", namespace, name, binding, prev.obj, user, "Binding")
        self._admit(a)
        self._validate_admission(a)
        old = prev.obj
        pod = dict(old)   # copy-on-write of exactly what apply_binding rewrites
        pod["metadata"] = dict(old["metadata"])
        if "annotations" in old["metadata"]:
            pod["metadata"]["annotations"] = dict(old["metadata"]["annotations"])
        pod["spec"] = dict(old.get("spec") or {})
        if pod["spec"].get("extendedResources"):
            pod["spec"]["extendedResources"] = [dict(r) for r in pod["spec"]["extendedResources"]]
        pod["status"] = dict(old.get("status") or {})
        if "conditions" in pod["status"]:
            pod["status"]["conditions"] = list(pod["status"]["conditions"])
        apply_binding(pod, binding)
        node = pod["spec"]["nodeName"]
        if self.store is not None:   # shared mode: the store enforces this with device claim keys
            idx = self.node_devices.get(node) or {}
            for rn, ids in core.pod_assigned_devices(pod).items():
                for i in ids:
                    owner = idx.get((rn, i))
                    if owner is not None and owner != key:
                        raise APIError(409, "Conflict", f"device {node}/{rn}/{i} is already assigned to {owner.rsplit('/', 2)[-2]}/{owner.rsplit('/', 1)[-1]}")
        return await self._commit(ri, key, MODIFIED, pod, prev)

    MAX_DISRUPTED_PODS = 2000          # eviction.go MaxDisruptedPodSize

    async def evict(self, namespace, name, eviction, user=None):
        """`pkg/registry/core/pod/storage/eviction.go`: an eviction is checked against the pod's
        PodDisruptionBudget and, when allowed, DECREMENTS it — disruptionsAllowed - 1 and the pod
        recorded in status.disruptedPods, written with the budget's resourceVersion (a conflict
        re-reads and re-checks), so concurrent evictions can never spend one disruption twice —
        before the pod is deleted. More than one matching budget is refused (500), as is a
        budget whose status the disruption controller has not caught up with (429)."""
        ri = m.BY_PLURAL["pods"]
        pod = (await self._aexisting(ri, namespace, name))[1].obj
        # pods/eviction is a CREATE of an Eviction through admission (NodeRestriction: a kubelet
        # evicts only its own pods), before the budget is touched
        ev = dict(eviction or {})
        ev.setdefault("metadata", {"name": name, "namespace": namespace})
        a = adm.Attributes(adm.CREATE, "pods", "eviction", namespace, name, ev, pod, user, "Eviction")
        self._admit(a)
        self._validate_admission(a)
        labels = (pod.get("metadata") or {}).get("labels") or {}
        from ..api.labels import label_selector_as_selector
        pri = m.BY_PLURAL["poddisruptionbudgets"]
        for attempt in range(8):
            pdbs = [p for p in self.list_objects("poddisruptionbudgets", namespace)
                    if label_selector_as_selector((p.get("spec") or {}).get("selector")).matches(labels)]
            if not pdbs:
                break
            if len(pdbs) > 1:
                raise APIError(500, "InternalError",
                               "This pod has more than one PodDisruptionBudget, which the eviction subresource does not support.")
            pdb = pdbs[0]
            st = dict(pdb.get("status") or {})
            too_many = APIError(429, "TooManyRequests", "Cannot evict pod as it would violate the pod's disruption budget.")
            if int(st.get("observedGeneration") or 0) < int(pdb["metadata"].get("generation") or 0):
                raise too_many
            allowed = st.get("disruptionsAllowed", st.get("podDisruptionsAllowed", 0)) or 0
            if allowed <= 0:
                raise too_many
            disrupted = dict(st.get("disruptedPods") or {})
            if len(disrupted) > self.MAX_DISRUPTED_PODS:
                raise APIError(403, "Forbidden", "DisruptedPods map too big - too many evictions not confirmed by PDB controller")
            disrupted[name] = now_rfc3339()
            st["disruptionsAllowed"] = allowed - 1
            st["disruptedPods"] = disrupted
            upd = dict(pdb, status=st)
            upd["metadata"] = dict(pdb["metadata"])
            try:
                await self.update(pri, namespace, m.name_of(pdb), upd, None, "status")
                break
            except APIError as e:
                if e.code != 409 or attempt == 7:
                    raise
                await asyncio.sleep(0)
        # the budget is spent: retry only the delete. A stale cache or a miss on this shared-store
        # worker must not bubble up to the request-level retry, which would re-run the whole
        # eviction and decrement the budget a second time (the reference retries only the
        # check-and-decrement, eviction.go:84-131)
        opts = (eviction or {}).get("deleteOptions") or {}
        return await self._retrying(lambda: self.delete(ri, namespace, name, opts, user))

    # ------------------------------------------------------------------
    # HTTP
    async def start(self, host="127.0.0.1", port=0, reuse_port=False):
        if self.remote_address and self.rstore is None:
            await self._start_remote()
        ctx = None
        cert, key, ca = self.tls
        if cert:
            import ssl
            ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
            ctx.load_cert_chain(cert, key)
            if ca:
                ctx.verify_mode = ssl.CERT_OPTIONAL    # x509 client-certificate authentication
                ctx.load_verify_locations(ca)
            if self.requestheader:
                ctx.verify_mode = ssl.CERT_OPTIONAL    # front-proxy client certificates
                ctx.load_verify_locations(self.requestheader["client_ca_file"])
        port = await self.http.start(host, port, ssl=ctx, reuse_port=reuse_port)
        await self._reconcile_master_endpoints("127.0.0.1" if host in ("0.0.0.0", "") else host, port)
        if self.event_ttl and self._reaper is None:
            self._reaper = asyncio.ensure_future(self._event_reaper())
        if self.compaction_interval > 0 and self._compactor is None:
            self._compactor = asyncio.ensure_future(self._compact_loop())
        return port

    async def _store_revision(self):
        return await self.rstore.revision() if self.rstore is not None else self.store.revision

    async def compact_to(self, rev):
        if rev <= 0:
            return
        if self.rstore is not None:
            await self.rstore.compact(rev)
        else:
            self.store.compact(rev)
        self.compactions += 1

    async def _compact_loop(self):
        prev = await self._store_revision()
        while True:
            await asyncio.sleep(self.compaction_interval)
            try:
                cur = await self._store_revision()
                await self.compact_to(prev)
                log.info("compacted storage history to revision %d", prev)
                prev = cur
            except Exception as e:  # noqa: BLE001 - the next pass retries
                log.warning("storage compaction failed: %s", e)

    async def start_insecure(self, host="127.0.0.1", port=0, reuse_port=False):
        """--insecure-port / --insecure-bind-address: plain HTTP with no authentication or
        authorization (requests run as system:unsecured in system:masters), served beside the
        secure port (`pkg/kubeapiserver/server/insecure_handler.go`)."""
        async def handler(req):
            req.insecure = True
            return await self._entry(req)
        self.insecure_http = HTTPServer(handler, request_timeout=self.request_timeout, long_running=self._long_running,
                                        timeout_response=_TIMEOUT_RESPONSE)
        self.insecure_port = await self.insecure_http.start(host, port, reuse_port=reuse_port)
        return self.insecure_port

    # long-running requests (`server/filters/longrunning.go`): no --request-timeout
    _LONG_RUNNING = frozenset(("proxy", "log", "exec", "attach", "portforward"))

    def _long_running(self, req):
        if req.query.get("watch") in ("true", "1") or "/watch/" in req.path or req.query.get("follow") in ("true", "1"):
            return True
        return any(seg in self._LONG_RUNNING for seg in req.path.split("/")) or \
            "upgrade" in req.headers.get("connection", "").lower()

    def _cors_headers(self, origin):
        if not any(r.search(origin) for r in self.cors):
            return None
        return {"Access-Control-Allow-Origin": origin,
                "Access-Control-Allow-Methods": "POST, GET, OPTIONS, PUT, DELETE, PATCH",
                "Access-Control-Allow-Headers": "Content-Type, Content-Length, Accept-Encoding, X-CSRF-Token, Authorization",
                "Access-Control-Expose-Headers": "Date", "Access-Control-Allow-Credentials": "true"}

    async def _entry(self, req):
        """HTTP entry with the CORS filter (the request timeout lives in the HTTP server)."""
        resp = await self.handle(req)
        if self.cors and req.headers.get("origin") and isinstance(resp, Response):
            extra = self._cors_headers(req.headers["origin"])
            if extra:
                resp.headers = dict(resp.headers or {}, **extra)
        return resp

    def expired_events(self, now=None):
        """Events whose last write (lastTimestamp, else creationTimestamp) is older than the TTL."""
        return self._expired([e.obj for e in list(self.caches["events"].by_key.values())], now)

    def _expired(self, events, now=None):
        now = time.time() if now is None else now
        out = []
        for o in events:
            t = parse_rfc3339(o.get("lastTimestamp")) or parse_rfc3339((o.get("metadata") or {}).get("creationTimestamp"))
            if t is not None and now - t > self.event_ttl:
                out.append(o)
        return out

    async def reap_events(self, now=None):
        n = 0
        ri = m.BY_PLURAL["events"]
        if "events" in self.uncached:
            entries, _ = await self._store_entries(ri)
            expired = self._expired([e.obj for e in entries], now)
        else:
            expired = self.expired_events(now)
        for o in expired:
            md = o["metadata"]
            try:
                await self._retrying(lambda md=md: self.delete(ri, md.get("namespace"), md["name"], {}))
                n += 1
            except APIError as e:
                if e.code not in (404, 409):       # another worker reaped it first
                    log.warning("event TTL delete of %s failed: %s", md["name"], e)
        return n

    async def _event_reaper(self):
        period = max(1.0, min(60.0, self.event_ttl / 4))
        while True:
            await asyncio.sleep(period)
            try:
                await self.reap_events()
            except Exception as e:  # noqa: BLE001 - keep reaping
                log.warning("event TTL reaper pass failed: %s", e)

    async def _reconcile_master_endpoints(self, ip, port):
        """Endpoints of the `kubernetes` service = the API servers (master-count reconciler: this
        server's advertise address joins the existing ones, at most --apiserver-count kept)."""
        if self.endpoint_reconciler == "none":
            return
        ip = self.advertise_address or ip
        cur = self.get_object("endpoints", "default", "kubernetes")
        addrs = [{"ip": ip}]
        if cur is not None and self.apiserver_count > 1:
            for ss in cur.get("subsets") or ():
                for a in ss.get("addresses") or ():
                    if a.get("ip") != ip and len(addrs) < self.apiserver_count:
                        addrs.append({"ip": a["ip"]})
        addrs.sort(key=lambda a: a["ip"])
        subsets = [{"addresses": addrs, "ports": [{"name": "https", "port": port, "protocol": "TCP"}]}]
        ri = m.BY_PLURAL["endpoints"]
        try:
            if cur is None:
                await self._retrying(lambda: self.create(ri, "default", {"metadata": {"name": "kubernetes", "namespace": "default"},
                                                                          "subsets": subsets}, admit=False))
            elif cur.get("subsets") != subsets:
                await self._retrying(lambda: self.guaranteed_update(ri, "default", "kubernetes",
                                                                    lambda o: o.__setitem__("subsets", subsets)))
        except APIError as e:
            if e.code != 409:
                log.warning("master endpoints reconcile failed: %s", e)

    async def stop(self):
        if self._reaper is not None:
            self._reaper.cancel()
            self._reaper = None
        if self._compactor is not None:
            self._compactor.cancel()
            self._compactor = None
        await self.http.stop()
        if self.insecure_http is not None:
            await self.insecure_http.stop()
        if self.rstore is not None:
            self.store_healthy = False   # a deliberate close, not a store failure
            await self.rstore.close()

    def _parse_path(self, path):
        """Returns (ri, namespace, name, subresource, watch) or a discovery/special marker."""
        parts = [p for p in path.split("/") if p]
        if not parts:
            return None
        if parts[0] == "api":
            if len(parts) == 1:
                return ("discovery", "api")
            if parts[1] != "v1":
                return None
            group, version, rest = "", "v1", parts[2:]
        elif parts[0] == "apis":
            if len(parts) == 1:
                return ("discovery", "apis")
            if len(parts) == 2:
                return ("discovery", "group", parts[1])
            group, version, rest = parts[1], parts[2], parts[3:]
        else:
            return None
        if group and self.aggregator.lookup(group, version) is not None and \
                not any(r.group == group and r.version == version for r in m.RESOURCES if r.plural in self.caches):
            return ("aggregated", self.aggregator.lookup(group, version))
        if not rest:
            return ("discovery", "resources", group, version)
        watch = False
        if rest[0] == "watch":
            watch = True
            rest = rest[1:]
        ns = None
        if rest[0] == "namespaces" and len(rest) >= 3 and not (len(rest) == 3 and rest[2] in ("status", "finalize")):
            ns = rest[1]
            rest = rest[2:]
        plural = rest[0]
        if plural == "componentstatuses" and group == "" and ns is None:
            return ("componentstatuses", rest[1] if len(rest) > 1 else None)
        ri = m.BY_PLURAL.get(plural)
        aliased = (group, version, plural) in m.ALIASES
        if ri is None or (ri.group != group and not aliased) or plural not in self.caches:
            if plural == "bindings" and ns:
                return ("bindings", ns)
            return None
        if ri.version != version and not aliased:
            return None
        if self.disabled_gv and (group, version) in self.disabled_gv or \
                self.disabled_res and (group, version, plural) in self.disabled_res:
            return None                 # --runtime-config switched it off
        name = rest[1] if len(rest) > 1 else None
        sub = "/".join(rest[2:]) if len(rest) > 2 else ""
        return (ri, ns, name, sub, watch)

    async def handle(self, req):
        t0 = time.perf_counter()
        verb = req.method
        resource = ""
        sub = ""
        code = 500
        try:
            p = req.path
            if p == "/healthz" or p.startswith("/healthz/") or p in ("/livez", "/readyz"):
                code = 200
                return Response(200, b"ok", "text/plain")
            if p == "/metrics":
                code = 200
                return Response(200, self.metrics.render(), "text/plain; version=0.0.4")
            if p == "/version":
                code = 200
                return _json(200, VERSION)
            if p.startswith("/debug/pprof") and self.enable_profiling:
                from ..utils.profiling import handle_debug
                resp = await handle_debug(req)
                code = resp.status
                return resp
            if self.cors and req.headers.get("origin"):
                cors = self._cors_headers(req.headers["origin"])
                if cors is not None and verb == "OPTIONS":
                    code = 204
                    return Response(204, b"", "text/plain", headers=cors)
            if p == "/logs" or p.startswith("/logs/"):
                if not self.enable_logs_handler:
                    code = 404
                    return _json(404, m.status_obj(404, "NotFound", "the server could not find the requested resource"))
            if p.rstrip("/") == "/swagger-ui" and self.enable_swagger_ui:
                code = 200
                return Response(200, SWAGGER_UI_PAGE, "text/html")
            user = ANONYMOUS
            if getattr(req, "insecure", False):
                user = UNSECURED
            elif self.authn is not None:
                ar = getattr(self.authn, "authenticate_request", None)
                if ar is not None and self._blocking_auth()[0]:
                    user = await asyncio.to_thread(ar, req)
                else:
                    user = ar(req) if ar is not None else self.authn.authenticate(req.headers)
                if user is None:
                    code = 401
                    return _json(401, m.status_obj(401, "Unauthorized", "Unauthorized"))
            if user is not UNSECURED and impersonation.requested(req.headers):
                try:
                    user = impersonation.impersonate(
                        req.headers, user, lambda u, verb, ns, res, sub, name, grp:
                        self._authorize(u, verb, ns, res, sub, name, grp, p))
                except impersonation.ImpersonationError as e:
                    code = e.code
                    return _json(e.code, m.status_obj(e.code, "BadRequest", e.message))
            req.user = user
            if p == "/logs" or p.startswith("/logs/"):
                await self._authz(user, "get", None, "", "", "", "", p, resource_request=False)
                from ..utils.httpserver import log_dir_response
                resp = log_dir_response(self.log_dir, p[len("/logs"):].lstrip("/"))
                code = resp.status
                return resp
            if p in ("/openapi/v2", "/swagger.json", "/swagger-2.0.0.json"):
                schemas = {}
                for plural, sch in self.crds.schemas.items():
                    ri = m.BY_PLURAL.get(plural)
                    if ri is not None and sch:
                        schemas[(ri.group, ri.version, ri.kind)] = sch
                code = 200
                return Response(200, self.openapi.get(schemas), "application/json")
            if req.body and req.headers.get("content-type", "").startswith(codec.PROTOBUF):
                # protobuf request bodies (`application/vnd.kubernetes.protobuf`, k8s\0 envelope):
                # decoded once, natively; handlers take the object (`_body`)
                try:
                    req.obj = pb.decode_object(req.body)
                except pb.ProtobufError as e:
                    raise APIError(415, "UnsupportedMediaType", str(e))
            if p.startswith("/api/v1/proxy/"):
                from .subresources import legacy_proxy_path
                p = legacy_proxy_path(p) or p
            parsed = self._parse_path(p)
            if parsed is None:
                code = 404
                return _json(404, m.status_obj(404, "NotFound", f"the server could not find the requested resource ({p})"))
            if parsed[0] == "discovery":
                code = 200
                return self._discovery(parsed)
            if parsed[0] == "aggregated":
                resp = await self.aggregator.proxy(req, parsed[1])
                code = resp.status
                return resp
            if parsed[0] == "componentstatuses":
                resource = "componentstatuses"
                await self._authz(user, "get" if parsed[1] else "list", None, "componentstatuses", "", parsed[1] or "", "", p)
                resp = await self._component_statuses(parsed[1])
                code = resp.status
                return resp
            if parsed[0] == "bindings":
                resource, sub = "pods", "binding"
                body = _body(req)
                await self._authz(user, "create", parsed[1], "pods", "binding", m.name_of(body), "", p)
                await self._retrying(lambda: self.bind(parsed[1], m.name_of(body), body, user))
                code = 201
                return _json(201, {"kind": "Status", "apiVersion": "v1", "metadata": {}, "status": "Success", "code": 201})
            ri, ns, name, sub, watch = parsed
            resource = ri.plural
            served = _requested_gv(p)
            if served != ri.group_version:
                # served under an alias group/version: store canonical, answer in the requested one
                req.served_gv = served
                if req.obj is not None:
                    if req.obj.get("apiVersion") == served:
                        req.obj["apiVersion"] = ri.group_version
                elif req.body and req.body[:1] == b"{":
                    try:
                        bo = codec.loads(req.body)
                        if bo.get("apiVersion") == served:
                            bo["apiVersion"] = ri.group_version
                            req.body = codec.dumpb(bo)
                    except ValueError:
                        pass
            is_watch = watch or req.query.get("watch") in ("true", "1")
            mutating = verb not in ("GET", "HEAD")
            # max-in-flight (filters/maxinflight.go WithMaxInFlightLimit): long-running requests
            # (watch, proxy, exec / attach / portforward / log — BasicLongRunningRequestCheck) are
            # not counted; a limit of 0 disables its budget; system:masters pass when over it
            long_running = is_watch or (sub or "").split("/")[0] in ("proxy", "exec", "attach", "portforward", "log")
            limited = False
            if not long_running:
                lim, cur, kind = ((self.max_mutating, self.inflight_mut, "mutating") if mutating
                                  else (self.max_inflight, self.inflight, "readOnly"))
                if lim and cur >= lim:
                    self.m_dropped.labels(kind).inc()
                    if "system:masters" not in (getattr(user, "groups", None) or ()):
                        code = 429
                        return Response(429, codec.dumpb(m.status_obj(429, "TooManyRequests",
                                                                      "Too many requests, please try again later.")),
                                        headers={"Retry-After": "1"})
                limited = True
            if ri.namespaced is False:
                ns = None
            if limited:                              # only budgeted requests are counted
                if mutating:
                    self.inflight_mut += 1
                else:
                    self.inflight += 1
            try:
                if self.rstore is not None and mutating:
                    # writes to one object through THIS worker queue up instead of racing on
                    # compare-and-swap; cross-worker races are resolved by _retrying
                    lock = None
                    if name is not None:
                        lk = (ri.plural, ns, name)
                        lock = self._key_locks.get(lk)
                        if lock is None:
                            lock = self._key_locks[lk] = asyncio.Lock()
                    try:
                        if lock is not None:
                            async with lock:
                                resp = await self._retrying(lambda: self._dispatch(req, ri, ns, name, sub, is_watch, user))
                        else:
                            resp = await self._retrying(lambda: self._dispatch(req, ri, ns, name, sub, is_watch, user))
                    finally:
                        if lock is not None and not lock.locked() and not lock._waiters:
                            self._key_locks.pop(lk, None)
                else:
                    resp = await self._dispatch(req, ri, ns, name, sub, is_watch, user)
            finally:
                if limited:
                    if mutating:
                        self.inflight_mut -= 1
                    else:
                        self.inflight -= 1
            code = getattr(resp, "status", 200)
            gv = getattr(req, "served_gv", None)
            if gv and isinstance(resp, Response) and resp.body[:1] == b"{" and code < 300:
                resp = Response(resp.status, _rewrite_gv(resp.body, ri.group_version, gv), resp.content_type)
            if verb == "GET" and code == 200 and isinstance(resp, Response) and resp.body[:1] == b"{" and \
                    "as=Table" in req.headers.get("accept", "") and not sub:
                from .subresources import to_table, wants_table
                if wants_table(req.headers["accept"]):
                    resp = _json(200, to_table(codec.loads(resp.body), ri.kind, q_include(req)))
                    return resp
            if codec.PROTOBUF in req.headers.get("accept", "") and isinstance(resp, Response) and resp.body[:1] == b"{":
                e = resp.entry
                if e is not None and gv in (None, ri.group_version) and pb.supported(ri.kind, ri.group_version):
                    # the cached object's envelope (the stored bytes + resourceVersion when this
                    # worker has them): no JSON decode, no re-encode from a dict
                    resp = Response(resp.status, e.pb_envelope(), codec.PROTOBUF)
                else:
                    obj = codec.loads(resp.body)
                    if pb.supported(obj.get("kind", "")):
                        resp = Response(resp.status, pb.encode_object(obj), codec.PROTOBUF)
            return resp
        except APIError as e:
            code = e.code
            return _err(e)
        except (ValueError, SelectorError) as e:
            code = 400
            return _json(400, m.status_obj(400, "BadRequest", str(e)))
        finally:
            self.m_requests.labels(verb, resource, sub, code).inc()
            if resource:
                dt = time.perf_counter() - t0
                self.m_latency.labels(verb, resource).observe(dt)
                if dt > 0.5 and verb != "GET":
                    # utiltrace LogIfLong (registry/store.go: 500 ms) for slow mutating calls
                    log.warning('Trace "%s %s" (code %s) total %.1f ms', verb, req.path, code, dt * 1e3)
            if self.audit is not None and resource:
                line = self.audit.log(req, verb, resource, sub, code)
                if line is not None and self.audit.blocking:
                    await self.audit.deliver(line)

    def _blocking_auth(self):
        """Webhook authenticators / authorizers answer over HTTP: their cache misses run off the
        event loop so one slow backend never stalls every other request."""
        flags = getattr(self, "_blocking_flags", None)
        if flags is None:
            from .auth import WebhookAuthorizer
            from .authn import WebhookTokenAuthenticator
            azs = getattr(self.authz, "authorizers", None) or [self.authz]
            toks = getattr(self.authn, "tok_auth", None) or ()
            flags = self._blocking_flags = (any(isinstance(t, WebhookTokenAuthenticator) for t in toks),
                                            any(isinstance(a, WebhookAuthorizer) for a in azs))
        return flags

    async def _authz(self, user, verb, ns, resource, sub, name, group, path, resource_request=True):
        if user is not UNSECURED and self._blocking_auth()[1]:
            return await asyncio.to_thread(self._authorize, user, verb, ns, resource, sub, name, group, path,
                                           resource_request)
        return self._authorize(user, verb, ns, resource, sub, name, group, path, resource_request)

    def _authorize(self, user, verb, ns, resource, sub, name, group, path, resource_request=True):
        if user is UNSECURED:
            return                  # the insecure port has no authorization
        ok, why = self.authz.authorize(AttributesRecord(user, verb, ns or "", resource, sub, name or "", group, path,
                                                        resource_request))
        if not ok:
            raise APIError(403, "Forbidden", why or "forbidden")

    # subresources this server serves; anything else under a named object is 404, never a write
    # of the request body to the object itself
    _SUBRESOURCES = frozenset(("", "status", "binding", "eviction", "log", "exec", "attach", "portforward",
                               "approval", "finalize", "scale", "rollback"))

    async def _dispatch(self, req, ri, ns, name, sub, is_watch, user):
        method = req.method
        q = req.query
        if sub:
            from . import subresources as sr
            if (sub == "proxy" or sub.startswith("proxy/")) and ri.plural in ("pods", "services", "nodes"):
                return await sr.handle_proxy(self, req, ri, ns, name, sub, user)
            if sub == "scale" and ri.plural in sr.SCALABLE:
                return await sr.handle_scale(self, req, ri, ns, name, user)
            if sub == "rollback" and ri.plural == "deployments" and method == "POST":
                return await sr.handle_rollback(self, req, ri, ns, name, user)
            if sub not in self._SUBRESOURCES or sub in ("scale", "rollback"):
                raise APIError(404, "NotFound", f"the server could not find the requested resource ({req.path})")
        if method in ("GET", "HEAD"):
            if is_watch:
                await self._authz(user, "watch", ns, ri.plural, sub, name, ri.group, req.path)
                return self._watch(req, ri, ns, name)
            if name is None:
                await self._authz(user, "list", ns, ri.plural, "", "", ri.group, req.path)
                if ri.plural in self.uncached:
                    return await self._list_store(req, ri, ns)
                return self._list(req, ri, ns)
            if sub == "log" and ri.plural == "pods":
                await self._authz(user, "get", ns, "pods", "log", name, "", req.path)
                return await self._pod_log(ns, name, q)
            if sub in ("exec", "attach", "portforward") and ri.plural == "pods":
                await self._authz(user, "get", ns, "pods", sub, name, "", req.path)
                return await self._pod_stream(req, ns, name, sub)
            await self._authz(user, "get", ns, ri.plural, sub, name, ri.group, req.path)
            if ri.plural in self.uncached:
                e = (await self._aexisting(ri, ns, name))[1]
            else:
                key = m.key_for(ri, ns, name)
                e = self.caches[ri.plural].get(key)
                if e is None and self.rstore is not None:
                    # shared mode: a miss may only mean this worker lags the writer — ask the store
                    _, e = await self._retrying(lambda: self._async_existing(ri, ns, name))
                if e is None:
                    raise not_found(ri, name)
            if q.get("export") in ("true", "1"):
                from .registry import export_object
                return _json(200, export_object(self.strategies[ri.plural], e.obj, q.get("exact") in ("true", "1")))
            return _entry_resp(req, ri, 200, e)
        body = req.body
        if method == "POST":
            if name is not None and sub == "binding" and ri.plural == "pods":
                await self._authz(user, "create", ns, "pods", "binding", name, "", req.path)
                await self.bind(ns, name, _body(req), user)
                return _json(201, {"kind": "Status", "apiVersion": "v1", "metadata": {}, "status": "Success", "code": 201})
            if name is not None and sub in ("exec", "attach", "portforward") and ri.plural == "pods":
                await self._authz(user, "create", ns, "pods", sub, name, "", req.path)
                return await self._pod_stream(req, ns, name, sub)
            if name is not None and sub == "eviction" and ri.plural == "pods":
                await self._authz(user, "create", ns, "pods", "eviction", name, "", req.path)
                await self.evict(ns, name, _body(req) if body else {}, user)
                return _json(201, {"kind": "Status", "apiVersion": "v1", "metadata": {}, "status": "Success", "code": 201})
            if name is not None:
                raise APIError(405, "MethodNotAllowed", "POST to a named resource is not allowed")
            if ri.plural in m.VIRTUAL:
                return self._review(ri, ns, _body(req), user, req)
            await self._authz(user, "create", ns, ri.plural, "", "", ri.group, req.path)
            obj = _body(req)
            if ri.namespaced and ns is None:
                ns = (obj.get("metadata") or {}).get("namespace") or "default"
            e = await self.create(ri, ns, obj, user)
            return _entry_resp(req, ri, 201, e)
        if name is None:
            if method == "DELETE":
                return await self._delete_collection(req, ri, ns, user)
            raise APIError(405, "MethodNotAllowed", f"{method} requires a name")
        if method == "PUT":
            if ri.plural == "namespaces" and sub == "finalize":
                await self._authz(user, "update", None, "namespaces", "finalize", name, "", req.path)
                return await self._finalize_namespace(name, _body(req), user)
            await self._authz(user, "update", ns, ri.plural, sub, name, ri.group, req.path)
            e = await self.update(ri, ns, name, _body(req), user, sub)
            return _entry_resp(req, ri, 200, e)
        if method == "PATCH":
            await self._authz(user, "patch", ns, ri.plural, sub, name, ri.group, req.path)
            e = await self.patch(ri, ns, name, req.headers.get("content-type", "application/merge-patch+json"), body, user, sub)
            return _entry_resp(req, ri, 200, e)
        if method == "DELETE":
            await self._authz(user, "delete", ns, ri.plural, "", name, ri.group, req.path)
            opts = _body(req) if body else {}
            if "gracePeriodSeconds" in q:
                opts["gracePeriodSeconds"] = int(q["gracePeriodSeconds"])
            if "propagationPolicy" in q:
                opts["propagationPolicy"] = q["propagationPolicy"]
            e, _ = await self.delete(ri, ns, name, opts, user)
            return _entry_resp(req, ri, 200, e)
        raise APIError(405, "MethodNotAllowed", f"method {method} not allowed")

    def _review(self, ri, ns, body, user, req):
        """TokenReview / SubjectAccessReview / SelfSubjectAccessReview / LocalSubjectAccessReview
        (`pkg/registry/authentication/tokenreview`, `pkg/registry/authorization/*`): answered by
        this server's authenticator / authorizer, never stored."""
        from .auth import User
        out = dict(body)
        out["kind"], out["apiVersion"] = ri.kind, ri.group_version
        out.setdefault("metadata", {})
        sp = body.get("spec") or {}
        if ri.plural == "tokenreviews":
            self._authorize(user, "create", None, ri.plural, "", "", ri.group, req.path)
            u = self.authn.authenticate({"authorization": f"Bearer {sp.get('token', '')}"}) if self.authn else None
            out["status"] = {"authenticated": u is not None}
            if u is not None:
                out["status"]["user"] = {"username": u.name, "uid": u.uid or "", "groups": list(u.groups)}
            return _json(201, out)
        if ri.plural == "selfsubjectaccessreviews":
            subj = user
        else:
            self._authorize(user, "create", ns, ri.plural, "", "", ri.group, req.path)
            subj = User(sp.get("user", ""), sp.get("uid", ""), list(sp.get("groups") or ()))
        ra = sp.get("resourceAttributes")
        nra = sp.get("nonResourceAttributes")
        if ra is not None:
            rns = ns if ri.plural == "localsubjectaccessreviews" else ra.get("namespace", "")
            rec = AttributesRecord(subj, ra.get("verb", ""), rns or "", ra.get("resource", ""), ra.get("subresource", ""),
                                   ra.get("name", ""), ra.get("group", ""), "", True)
        elif nra is not None:
            rec = AttributesRecord(subj, (nra.get("verb") or "get").lower(), "", "", "", "", "", nra.get("path", ""), False)
        else:
            raise bad_request("spec.resourceAttributes or spec.nonResourceAttributes is required")
        ok, why = self.authz.authorize(rec)
        out["status"] = {"allowed": bool(ok)}
        if why:
            out["status"]["reason"] = why
        return _json(201, out)

    async def _finalize_namespace(self, name, obj, user):
        ri = m.BY_PLURAL["namespaces"]
        key, prev = self._existing(ri, None, name)
        new = fast_copy(prev.obj)
        new.setdefault("spec", {})["finalizers"] = list((obj.get("spec") or {}).get("finalizers") or [])
        if new["metadata"].get("deletionTimestamp") and not new["spec"]["finalizers"] and not new["metadata"].get("finalizers"):
            e = await self._commit(ri, key, DELETED, new, prev)
        else:
            e = await self._commit(ri, key, MODIFIED, new, prev)
        return Response(200, e.raw)

    async def _delete_collection(self, req, ri, ns, user):
        await self._authz(user, "deletecollection", ns, ri.plural, "", "", ri.group, req.path)
        ls = parse_labels(req.query.get("labelSelector")) if req.query.get("labelSelector") else None
        fs = parse_field_selector(req.query.get("fieldSelector")) if req.query.get("fieldSelector") else None
        opts = codec.loads(req.body) if req.body else {}
        if ri.plural in self.uncached:
            entries = (await self._store_entries(ri, ns, ls, fs))[0]
        else:
            entries = self.caches[ri.plural].list(m.prefix_for(ri, ns), ls, fs)
        # `DeleteCollection` of registry/generic/registry/store.go: --delete-collection-workers
        # goroutines take items off a shared queue; results keep the listing order
        results = [None] * len(entries)
        nxt = iter(range(len(entries)))

        async def worker():
            for i in nxt:
                e = entries[i]
                try:
                    d, _ = await self.delete(ri, m.namespace_of(e.obj) or None, m.name_of(e.obj), opts, user)
                    results[i] = d.obj
                except APIError as err:
                    if err.code != 404:
                        raise
        await asyncio.gather(*(worker() for _ in range(min(self.delete_collection_workers, len(entries)) or 1)))
        items = [o for o in results if o is not None]
        return _json(200, {"kind": ri.list_kind, "apiVersion": ri.group_version,
                           "metadata": {"resourceVersion": str(self.revision)}, "items": items})

    def _hide_uninitialized(self, q, fsel):
        if not self.initializers_enabled or q.get("includeUninitialized") in ("true", "1"):
            return fsel
        from .cacher import UNINITIALIZED
        return (fsel + "," if fsel else "") + f"{UNINITIALIZED}!=true"

    def _list(self, req, ri, ns):
        q = req.query
        ls = parse_labels(q.get("labelSelector")) if q.get("labelSelector") else None
        fsel = self._hide_uninitialized(q, q.get("fieldSelector"))
        fs = parse_field_selector(fsel) if fsel else None
        entries = self._shard_filter(q, self.caches[ri.plural].list(m.prefix_for(ri, ns), ls, fs))
        return self._list_response(q, ri, entries, str(self.revision))

    @staticmethod
    def _shard(q):
        v = q.get(QUERY_PARAM)
        return parse_shard(v) if v else None

    def _shard_filter(self, q, entries):
        sh = self._shard(q)
        if sh is None:
            return entries
        return [e for e in entries if shard_matches(e.fields, e.labels, *sh)]

    async def _list_store(self, req, ri, ns):
        q = req.query
        ls = parse_labels(q.get("labelSelector")) if q.get("labelSelector") else None
        fsel = self._hide_uninitialized(q, q.get("fieldSelector"))
        fs = parse_field_selector(fsel) if fsel else None
        entries, rev = await self._store_entries(ri, ns, ls, fs)
        return self._list_response(q, ri, self._shard_filter(q, entries), str(rev))

    def _list_response(self, q, ri, entries, rv):
        limit = int(q.get("limit") or 0)
        cont = q.get("continue")
        next_token = None
        if cont:
            try:
                tok = codec.loads(base64.urlsafe_b64decode(cont.encode()))
                start = tok["start"]
                rv = tok.get("rv", rv)
            except Exception:
                raise bad_request("continue key is not valid")
            entries = [e for e in entries if e.sort_key > start]
        if limit and len(entries) > limit:
            entries = entries[:limit]
            next_token = base64.urlsafe_b64encode(codec.dumpb({"rv": rv, "start": entries[-1].sort_key})).decode()
        md = '"resourceVersion":"%s"' % rv
        if next_token:
            md += ',"continue":"%s"' % next_token
        body = b'{"kind":"%s","apiVersion":"%s","metadata":{%s},"items":[' % (
            ri.list_kind.encode(), ri.group_version.encode(), md.encode()) + b",".join(e.raw for e in entries) + b"]}"
        return Response(200, body)

    def _fanout_spec(self, req, ri, ns, label_selector, field_selector, shard=None):
        """Requirements for kamd-etcd's watch fan-out, or None when this watch must stay here:
        TLS connections (the TLS session lives in this process), encrypted storage (the store
        cannot read the sealed index frame), quantity comparisons in label selectors. Protobuf
        values are transcoded to JSON by the store (native/pbcodec/pb_codec.h)."""
        if self.fanout is None or ri.plural in self.transformers:
            return None
        if req.transport is None or req.transport.get_extra_info("sslcontext") is not None:
            return None
        reqs = []
        if label_selector:
            for r in parse_labels(label_selector).reqs:
                op = {"=": "=", "==": "=", "!=": "!=", "in": "in", "notin": "notin", "exists": "exists", "!": "!"}.get(r.op)
                if op is None:
                    return None
                reqs.append((0, op, r.key, list(r.values)))
        if field_selector:
            for k, op, v in parse_field_selector(field_selector).terms:
                reqs.append((1, "!=" if op == "!=" else "=", k, [v]))
        if shard is not None:
            reqs.append((0, "shard", SHARD_OFFSET_LABEL, [shard[1], shard[0]]))
        return reqs

    @staticmethod
    def _wants_pb_watch(req, ri):
        """Content negotiation of a watch (`negotiation.NegotiateOutputStreamSerializer`): the
        first media type of the Accept header this server streams decides; protobuf only for
        kinds in the protobuf schema, served in their storage group/version."""
        accept = req.headers.get("accept", "")
        if "protobuf" not in accept:
            return False
        for part in accept.split(","):
            mt = part.split(";", 1)[0].strip().lower()
            if mt == codec.PROTOBUF:
                gv = getattr(req, "served_gv", None)
                return (gv is None or gv == ri.group_version) and pb.supported(ri.kind, ri.group_version)
            if mt in (codec.JSON, "*/*", "application/*"):
                return False
        return False

    def _watch_store(self, ri, ns, label_selector, field_selector, rv, timeout, shard=None, protobuf=False):
        """Watch of an uncached resource that the store's fan-out cannot serve (a TLS client,
        quantity label selectors): a store watch of its own, filtered here. Without the previous
        object state, a change that leaves the selector is reported as DELETED even if the
        client never had the object (informers ignore unknown deletes)."""
        from ..storage.etcd3_client import connect_store
        ls = parse_labels(label_selector) if label_selector else None
        fs = parse_field_selector(field_selector) if field_selector else None
        prefix = m.prefix_for(ri, ns if ri.namespaced else None)
        server = self

        def ok(e):
            return (ls is None or ls.matches(e.labels)) and (fs is None or fs.matches(e.fields)) and \
                (shard is None or shard_matches(e.fields, e.labels, *shard))

        def ev(t, e):
            return pb_event_bytes(t, e) if protobuf else event_bytes(t, e.raw)

        async def run(writer):
            st = await connect_store(server.remote_address, server.etcd_tls)
            done = asyncio.get_running_loop().create_future()
            seen: dict = {}
            try:
                if not rv or rv == "0":
                    kvs, _, frm = await st.range(prefix)
                    for kv in kvs:
                        e = server._entry_from_kv(ri.plural, kv)
                        if ok(e):
                            seen[kv.key] = True
                            writer.write(ev(ADDED, e))
                else:
                    frm = int(rv)

                def on_event(t, kv):
                    if t is None:
                        if not done.done():
                            done.set_result(None)
                        return
                    if t == wire.PROGRESS:
                        return
                    e = server._entry_from_kv(ri.plural, kv)
                    cur = t != wire.OP_DELETE and ok(e)
                    was = seen.get(kv.key, kv.version > 1 or t == wire.OP_DELETE)
                    if t == wire.OP_DELETE:
                        if was or ok(e):
                            writer.write(ev(DELETED, e))
                        seen.pop(kv.key, None)
                    elif cur:
                        writer.write(ev(MODIFIED if was and kv.version > 1 else ADDED, e))
                        seen[kv.key] = True
                    elif was:
                        writer.write(ev(DELETED, e))
                        seen[kv.key] = False
                try:
                    await st.watch(prefix, frm, on_event)
                except CompactedError:
                    writer.write(error_event(m.status_obj(410, "Expired", f"too old resource version: {frm}"), protobuf))
                    return
                server.m_watchers.labels(ri.kind).inc()
                try:
                    waits = [done, asyncio.ensure_future(writer.wait_closed())]
                    await asyncio.wait(waits, timeout=timeout, return_when=asyncio.FIRST_COMPLETED)
                    waits[1].cancel()
                finally:
                    server.m_watchers.labels(ri.kind).dec()
            finally:
                await st.close()

        return StreamResponse(run, pb.WATCH_STREAM if protobuf else "application/json")

    def _watch(self, req, ri, ns, name):
        q = req.query
        rv = q.get("resourceVersion")
        fsel = q.get("fieldSelector")
        if name:
            fsel = (fsel + "," if fsel else "") + f"metadata.name={name}"
        fsel = self._hide_uninitialized(q, fsel)
        timeout = float(q.get("timeoutSeconds") or 0) or None
        if timeout is None and self.min_request_timeout:
            # `watch.go` serveWatch: timeout = minRequestTimeout * (1 + rand) when unspecified
            import random
            timeout = self.min_request_timeout * (1.0 + random.random())
        shard = self._shard(q)
        protobuf = self._wants_pb_watch(req, ri)
        reqs = self._fanout_spec(req, ri, ns, q.get("labelSelector"), fsel, shard)
        if reqs is not None:
            # shared-store mode: the store streams this watch itself (C++ fan-out), JSON lines or
            # protobuf frames
            send_initial = not rv or rv == "0"
            msg = self.fanout.encode(m.prefix_for(ri, ns), send_initial, 0 if send_initial else int(rv), timeout, reqs,
                                     protobuf=protobuf)
            self.m_fanout.labels(ri.plural).inc()
            return HandoffResponse(lambda fd: self.fanout.handoff(fd, msg))
        if ri.plural in self.uncached:
            return self._watch_store(ri, ns, q.get("labelSelector"), fsel, rv, timeout, shard, protobuf)
        cache = self.caches[ri.plural]
        send_initial = not rv or rv == "0"
        from_rev = int(rv) if rv and rv != "0" else None
        if from_rev is not None and cache.events and from_rev < cache.events[0][0] - 1 \
                and len(cache.events) == cache.events.maxlen:
            raise APIError(410, "Expired", f"too old resource version: {from_rev} ({cache.events[0][0] - 1})")
        server = self

        async def run(writer):
            try:
                w = cache.add_watcher(writer, ns, q.get("labelSelector"), fsel, from_rev, send_initial, shard, protobuf)
            except GoneError as e:
                writer.write(error_event(m.status_obj(410, "Expired", str(e)), protobuf))
                return
            server.m_watchers.labels(ri.kind).inc()
            try:
                fut = writer.wait_closed()
                if timeout:
                    await asyncio.wait_for(asyncio.shield(fut), timeout)
                else:
                    await fut
            except asyncio.TimeoutError:
                pass
            finally:
                w.stop()
                server.m_watchers.labels(ri.kind).dec()

        return StreamResponse(run, pb.WATCH_STREAM if protobuf else "application/json")

    async def _kubelet_of(self, ns, name):
        """(pod, kubelet host, kubelet port) — the node connection info the reference resolves in
        `pkg/registry/core/pod/strategy.go` ResourceLocation / streamLocation."""
        if "pods" in self.uncached:
            pod = (await self._aexisting(m.BY_PLURAL["pods"], ns, name))[1].obj
        else:
            pod = self.get_object("pods", ns, name)
            if pod is None:
                raise not_found(m.BY_PLURAL["pods"], name)
        node = (pod.get("spec") or {}).get("nodeName")
        if not node:
            raise bad_request(f"pod {name} is not scheduled")
        nobj = self.get_object("nodes", None, node)
        port = ((nobj or {}).get("status") or {}).get("daemonEndpoints", {}).get("kubeletEndpoint", {}).get("Port") \
            or (self.kubelet_port if nobj is not None else None)
        addr = node_address(nobj, self.kubelet_address_types)
        if not port:
            raise APIError(503, "ServiceUnavailable", f"node {node} has no kubelet endpoint")
        return pod, addr, port

    async def _pod_stream(self, req, ns, name, sub):
        """pods/exec, pods/attach and pods/portforward proxied to the node's kubelet: WebSocket
        upgrades are relayed as-is (channel.k8s.io protocols), the framed stream / `Upgrade: tcp`
        fallback is re-framed (`pkg/registry/core/pod/rest/subresources.go` ExecREST/PortForwardREST)."""
        from urllib.parse import parse_qs, urlencode
        pod, addr, port = await self._kubelet_of(ns, name)
        a = adm.Attributes(adm.CONNECT, "pods", sub, ns, name, None, pod, getattr(req, "user", None), "Pod")
        self._admit(a)
        self._validate_admission(a)
        q = parse_qs(req.qs or "")
        from ..cri.remotecommand import is_upgrade_request
        if is_upgrade_request(req.headers):
            # UpgradeAwareHandler: relay the WebSocket / SPDY upgrade to the kubelet and splice
            from ..cri.remotecommand import upgrade_proxy_response
            kb = f"{self.kubelet_scheme}://{addr}:{port}"
            if sub == "portforward":
                return upgrade_proxy_response(req, f"{kb}/portForward/{ns}/{name}?{req.qs}", ssl_context=self.kubelet_ssl)
            containers = (pod.get("spec") or {}).get("containers") or [{}]
            cname = (q.get("container") or [containers[0].get("name", "")])[0]
            return upgrade_proxy_response(req, f"{kb}/{sub}/{ns}/{name}/{cname}?{req.qs}", ssl_context=self.kubelet_ssl)
        if sub == "portforward":
            pport = (q.get("port") or q.get("ports") or [""])[0]
            if not pport:
                raise bad_request("port is required")
            if "upgrade" not in req.headers.get("connection", "").lower():
                raise bad_request("port-forward needs Connection: Upgrade")
            from ..cri.server import splice
            from ..cri.streaming import open_port_forward
            url = f"{self.kubelet_scheme}://{addr}:{port}/portForward/{ns}/{name}"

            async def run(reader, writer):
                ur, uw = await open_port_forward(url, int(pport), ssl_context=self.kubelet_ssl)
                await splice(reader, writer, ur, uw)
            return UpgradeResponse(run)
        containers = (pod.get("spec") or {}).get("containers") or [{}]
        cname = (q.get("container") or [containers[0].get("name", "")])[0]
        names = {c.get("name") for c in containers} | {c.get("name") for c in (pod.get("spec") or {}).get("initContainers") or ()}
        if cname not in names:
            raise bad_request(f"container {cname} is not valid for pod {name}")
        target = f"{self.kubelet_scheme}://{addr}:{port}/{sub}/{ns}/{name}/{cname}"
        if q.get("command"):
            target += "?" + urlencode([("command", c) for c in q["command"]])
        from ..cri.streaming import _open

        async def relay(w):
            r, uw, status, _ = await _open(target, ssl_context=self.kubelet_ssl)
            try:
                if status != 200:
                    body = await r.read(4096)
                    msg = b"\x01" + body
                    w.transport.write(b"%x\r\n%s\r\n" % (len(msg), msg))
                    w.transport.write(b"2\r\n\x03" + b"1" + b"\r\n")
                    return
                while True:
                    line = await r.readuntil(b"\r\n")
                    size = int(line.strip(), 16)
                    if size == 0:
                        break
                    w.transport.write(line + await r.readexactly(size + 2))
            finally:
                uw.close()
        return StreamResponse(relay, "application/vnd.kamd.stream")

    async def _component_statuses(self, name=None):
        """`pkg/registry/core/componentstatus/rest.go`: probe the scheduler, the controller
        manager and the store; one ComponentStatus each with a Healthy condition."""
        from ..client.http import HTTPClient

        async def probe(comp, url):
            if url is None:
                try:
                    if self.rstore is not None:
                        # shared / etcd store: it must answer, and this worker's watch be alive
                        await asyncio.wait_for(self.rstore.revision(), 1.5)
                        ok = self.store_healthy
                    else:
                        ok = self.store is not None
                    msg = '{"health": "true"}' if ok else "no store"
                except Exception as e:  # noqa: BLE001
                    ok, msg = False, str(e) or type(e).__name__
            else:
                base, _, path = url.partition("/healthz")
                c = HTTPClient(base, timeout=1.0)
                try:
                    st, body = await asyncio.wait_for(c.request("GET", "/healthz" + path), 1.5)
                    ok, msg = st == 200, body.decode(errors="replace")
                except (OSError, ConnectionError, asyncio.TimeoutError, ValueError) as e:
                    ok, msg = False, f"Get {url}: {e or type(e).__name__}"
                finally:
                    await c.close()
            cond = {"type": "Healthy", "status": "True" if ok else "False", "message": msg if ok else ""}
            if not ok:
                cond["error"] = msg
            return {"kind": "ComponentStatus", "apiVersion": "v1", "metadata": {"name": comp}, "conditions": [cond]}
        targets = dict(self.component_endpoints)
        targets.setdefault("etcd-0", None)
        if name is not None:
            if name not in targets:
                raise APIError(404, "NotFound", f'componentstatuses "{name}" not found')
            return _json(200, await probe(name, targets[name]))
        items = await asyncio.gather(*(probe(k, v) for k, v in sorted(targets.items())))
        return _json(200, {"kind": "ComponentStatusList", "apiVersion": "v1", "metadata": {}, "items": list(items)})

    async def _pod_log(self, ns, name, q):
        """pods/log relayed to the kubelet (`pkg/registry/core/pod/rest/log.go`); with follow the
        kubelet's stream is relayed as it arrives."""
        from urllib.parse import urlencode
        pod, addr, port = await self._kubelet_of(ns, name)
        q = dict(q)
        q["container"] = _log_container(pod, q.get("container", ""))
        from ..client.http import HTTPClient
        c = HTTPClient(f"{self.kubelet_scheme}://{addr}:{port}", ssl_context=self.kubelet_ssl,
                       timeout=max(self.kubelet_timeout, 30.0))
        qs = urlencode(q)
        path = f"/containerLogs/{ns}/{name}/{q.get('container', '')}" + (f"?{qs}" if qs else "")
        if q.get("follow") in ("true", "1"):
            st, hdrs, r, w = await c.open_raw("GET", path)
            if st != 200:
                body = await r.read(1 << 16)
                w.close()
                await c.close()
                return Response(st, body, "text/plain")

            async def relay(cw):
                try:
                    if hdrs.get("transfer-encoding", "").lower() == "chunked":
                        while True:
                            n = int((await r.readuntil(b"\r\n")).split(b";")[0].strip() or b"0", 16)
                            if n == 0:
                                return
                            cw.write(await r.readexactly(n))
                            await r.readexactly(2)
                    while True:
                        chunk = await r.read(1 << 16)
                        if not chunk:
                            return
                        cw.write(chunk)
                except (asyncio.IncompleteReadError, ConnectionError):
                    return
                finally:
                    w.close()
                    await c.close()
            return StreamResponse(relay, "text/plain")
        try:
            st, body = await c.request("GET", path)
        finally:
            await c.close()
        return Response(st, body, "text/plain")

    def _discovery(self, parsed):
        kind = parsed[1]
        if kind == "api":
            if ("", "v1") in self.disabled_gv:
                return _json(200, {"kind": "APIVersions", "versions": [], "serverAddressByClientCIDRs": []})
            return _json(200, {"kind": "APIVersions", "versions": ["v1"],
                               "serverAddressByClientCIDRs": [{"clientCIDR": "0.0.0.0/0", "serverAddress": "127.0.0.1"}]})
        groups = {g: {v for v in vs if (g, v) not in self.disabled_gv} for g, vs in m.served_versions().items() if g}
        groups = {g: vs for g, vs in groups.items() if vs}
        for g, vs in self.aggregator.groups().items():
            groups.setdefault(g, set()).update(vs)

        def ordered(vs):   # preferred (highest priority) first, as the reference lists them
            return sorted(vs, key=m.version_priority, reverse=True)
        if kind == "apis":
            return _json(200, {"kind": "APIGroupList", "apiVersion": "v1", "groups": [
                {"name": g, "versions": [{"groupVersion": f"{g}/{v}", "version": v} for v in ordered(vs)],
                 "preferredVersion": {"groupVersion": f"{g}/{ordered(vs)[0]}", "version": ordered(vs)[0]}}
                for g, vs in sorted(groups.items())]})
        if kind == "group":
            g = parsed[2]
            if g not in groups:
                raise APIError(404, "NotFound", f"group {g} not found")
            vs = ordered(groups[g])
            return _json(200, {"kind": "APIGroup", "apiVersion": "v1", "name": g,
                               "versions": [{"groupVersion": f"{g}/{v}", "version": v} for v in vs],
                               "preferredVersion": {"groupVersion": f"{g}/{vs[0]}", "version": vs[0]}})
        group, version = parsed[2], parsed[3]
        res = []
        if (group, version) in self.disabled_gv:
            raise APIError(404, "NotFound", f"{group}/{version} not found")
        for ri in m.RESOURCES:
            if not ((ri.group == group and ri.version == version) or (group, version, ri.plural) in m.ALIASES):
                continue
            if (group, version, ri.plural) in self.disabled_res:
                continue
            verbs = ["create", "delete", "deletecollection", "get", "list", "patch", "update", "watch"]
            res.append({"name": ri.plural, "singularName": "", "namespaced": ri.namespaced, "kind": ri.kind,
                        "verbs": verbs, "shortNames": list(ri.short)})
            if self.strategies[ri.plural].has_status:
                res.append({"name": ri.plural + "/status", "singularName": "", "namespaced": ri.namespaced,
                            "kind": ri.kind, "verbs": ["get", "patch", "update"]})
            if ri.plural in ("deployments", "replicasets", "statefulsets", "replicationcontrollers"):
                sgv = "autoscaling/v1" if ri.plural == "replicationcontrollers" or \
                    f"{group}/{version}" not in ("extensions/v1beta1", "apps/v1beta1", "apps/v1beta2") else f"{group}/{version}"
                res.append({"name": ri.plural + "/scale", "singularName": "", "namespaced": True, "group": sgv.split("/")[0],
                            "version": sgv.split("/")[1], "kind": "Scale", "verbs": ["get", "patch", "update"]})
            if ri.plural == "deployments" and f"{group}/{version}" in ("extensions/v1beta1", "apps/v1beta1"):
                res.append({"name": "deployments/rollback", "singularName": "", "namespaced": True,
                            "kind": "DeploymentRollback", "verbs": ["create"]})
            if ri.plural in ("pods", "services", "nodes"):
                res.append({"name": ri.plural + "/proxy", "singularName": "", "namespaced": ri.namespaced,
                            "kind": ri.kind + "ProxyOptions", "verbs": ["create", "delete", "get", "patch", "update"]})
            if ri.plural == "pods":
                res.append({"name": "pods/binding", "singularName": "", "namespaced": True, "kind": "Binding", "verbs": ["create"]})
                res.append({"name": "pods/eviction", "singularName": "", "namespaced": True, "kind": "Eviction", "verbs": ["create"]})
                res.append({"name": "pods/log", "singularName": "", "namespaced": True, "kind": "Pod", "verbs": ["get"]})
                for sr in ("exec", "attach", "portforward"):
                    res.append({"name": f"pods/{sr}", "singularName": "", "namespaced": True,
                                "kind": "PodExecOptions" if sr != "portforward" else "PodPortForwardOptions",
                                "verbs": ["create", "get"]})
        if group == "" and version == "v1":
            res.append({"name": "componentstatuses", "singularName": "", "namespaced": False, "kind": "ComponentStatus",
                        "verbs": ["get", "list"], "shortNames": ["cs"]})
        if not res:
            raise APIError(404, "NotFound", f"{group}/{version} not found")
        gv = f"{group}/{version}" if group else version
        return _json(200, {"kind": "APIResourceList", "groupVersion": gv, "resources": res})
