"""kube-apiserver entry point (reference: cmd/kube-apiserver/app/server.go:102-132).

    python -m kubernetes_amd.cmd.apiserver --port 8080                  # one process, embedded store
    python -m kubernetes_amd.cmd.apiserver --port 8080 --workers 4      # kamd-etcd + 4 worker processes
    python -m kubernetes_amd.cmd.apiserver --etcd-servers unix:///run/kamd-etcd.sock   # join a store

With `--workers N` (N > 1) this process becomes a supervisor: it starts the native store
(`kamd-etcd`, optionally with a WAL) and N API server worker processes that all listen on the
same port (SO_REUSEPORT — the kernel spreads client connections over them), the way several
kube-apiserver replicas sit in front of one etcd. If any child dies, the supervisor stops all
of them and exits non-zero.
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time

from ..api import codec
from ..apiserver.server import APIServer
from ..storage.mvcc import MVCCStore
from ._common import check_unsupported, deprecated_noop, run_until_signal, setup_logging, unsupported, write_port_file


def _parser():
    ap = argparse.ArgumentParser("kube-apiserver")
    ap.add_argument("--bind-address", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8080)
    ap.add_argument("--port-file", default=None, help="write the bound port here (use with --port 0)")
    ap.add_argument("--admission-control", default=None, help="comma separated ordered plugin list")
    ap.add_argument("--feature-gates", default="", help="e.g. PodPriority=true,ExpandPersistentVolumes=true")
    ap.add_argument("--admission-control-config-file", default=None,
                    help="AdmissionConfiguration: plugins[{name, path | configuration}]")
    ap.add_argument("--authorization-mode", default="AlwaysAllow")
    ap.add_argument("--token-auth-file", default=None)
    # the reference stores protobuf by default (cmd/kube-apiserver/app/options/options.go:117)
    ap.add_argument("--storage-media-type", default=codec.PROTOBUF)
    ap.add_argument("--storage-engine", default="native", choices=["native", "python"])
    ap.add_argument("--etcd-wal", default=None, help="durable WAL path for the store")
    ap.add_argument("--etcd-fan-threads", type=int, default=0,
                    help="watch fan-out threads of the shared native store (0 = KAMD_ETCD_FAN_THREADS or 1)")
    ap.add_argument("--etcd-servers", default=None,
                    help="the store: an etcd v3 cluster (comma-separated http(s)://HOST:PORT endpoints) or the "
                         "shared native store (unix://PATH or tcp://HOST:PORT)")
    ap.add_argument("--workers", type=int, default=1, help="API server worker processes sharing one native store")
    ap.add_argument("--reuse-port", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--max-requests-inflight", type=int, default=4000)
    ap.add_argument("--max-mutating-requests-inflight", type=int, default=2000)
    ap.add_argument("--watch-cache-size", type=int, default=200000)
    ap.add_argument("--event-ttl", default="1h", help="amount of time to retain events (e.g. 1h, 30m, 90s)")
    ap.add_argument("--audit-log-path", default=None, help="write audit events (JSON lines) here; '-' = stdout")
    ap.add_argument("--audit-policy-file", default=None, help="audit policy YAML (rules: level/users/verbs/resources)")
    ap.add_argument("--experimental-encryption-provider-config", dest="encryption_config", default=None,
                    help="EncryptionConfig YAML: encrypt the listed resources at rest (aescbc/aesgcm/secretbox/kms)")
    ap.add_argument("--kubelet-https", type=lambda v: v.lower() != "false", default=True,
                    help="use https for kubelet connections (logs, exec/attach/port-forward, node proxy)")
    ap.add_argument("--kubelet-certificate-authority", default=None,
                    help="CA that signs kubelet serving certificates (unset: they are not verified)")
    ap.add_argument("--kubelet-client-certificate", default=None, help="client certificate presented to kubelets")
    ap.add_argument("--kubelet-client-key", default=None)
    ap.add_argument("--tls-cert-file", default=None)
    ap.add_argument("--tls-private-key-file", default=None)
    ap.add_argument("--client-ca-file", default=None, help="enable x509 client certificate authentication")
    ap.add_argument("--service-account-key-file", action="append", default=[])
    ap.add_argument("--service-account-lookup", type=lambda v: v.lower() != "false", default=True)
    ap.add_argument("--enable-bootstrap-token-auth", action="store_true")
    ap.add_argument("--authentication-token-webhook-url", default=None)
    ap.add_argument("--anonymous-auth", type=lambda v: v.lower() != "false", default=True)
    ap.add_argument("--authorization-policy-file", default=None, help="ABAC policy (JSON lines)")
    ap.add_argument("--authorization-webhook-url", default=None)
    ap.add_argument("--service-cluster-ip-range", default="10.0.0.0/24")
    ap.add_argument("--service-node-port-range", default="30000-32767")
    ap.add_argument("--oidc-issuer-url", default=None)
    ap.add_argument("--oidc-client-id", default=None)
    ap.add_argument("--oidc-username-claim", default="sub")
    ap.add_argument("--oidc-username-prefix", default=None)
    ap.add_argument("--oidc-groups-claim", default=None)
    ap.add_argument("--oidc-groups-prefix", default="")
    ap.add_argument("--oidc-ca-file", default=None)
    ap.add_argument("--oidc-required-claim", action="append", default=[], help="key=value")
    ap.add_argument("--audit-webhook-config-file", default=None, help="kubeconfig naming the audit webhook")
    ap.add_argument("--audit-webhook-batch-max-size", type=int, default=400)
    ap.add_argument("--audit-webhook-batch-max-wait", type=float, default=1.0)
    _reference_flags(ap)
    ap.add_argument("-v", type=int, default=0)
    return ap


def load_admission_config(path):
    """`apiserver.k8s.io/v1alpha1 AdmissionConfiguration` → {plugin name: config dict}
    (`staging/src/k8s.io/apiserver/pkg/admission/config.go`: `configuration` inline or `path`
    to a file, relative to the admission config's directory)."""
    import yaml
    with open(path) as f:
        doc = yaml.safe_load(f) or {}
    out = {}
    for p in doc.get("plugins") or ():
        cfg = p.get("configuration")
        if cfg is None and p.get("path"):
            fp = p["path"] if os.path.isabs(p["path"]) else os.path.join(os.path.dirname(os.path.abspath(path)), p["path"])
            with open(fp) as f:
                cfg = yaml.safe_load(f)
        out[p["name"]] = cfg or {}
    return out


# flags the multi-worker supervisor sets itself for each worker
_SUPERVISOR_OWNED = {"workers", "port", "port_file", "etcd_wal", "etcd_fan_threads", "etcd_servers", "reuse_port", "bind_address",
                     "audit_log_path", "audit_policy_file", "v"}


def passthrough_args(a, parser=None):
    """Every explicitly set flag except the supervisor-owned ones, re-rendered for a worker."""
    parser = parser or _parser()
    out = []
    for act in parser._actions:  # noqa: SLF001 - argparse has no public action list
        if not act.option_strings or act.dest in _SUPERVISOR_OWNED or act.dest == "help":
            continue
        v = getattr(a, act.dest, None)
        if v == act.default or v is None:
            continue
        flag = act.option_strings[-1]
        if isinstance(act, argparse._StoreTrueAction):  # noqa: SLF001
            out.append(flag)
        elif isinstance(v, list):
            for x in v:
                out += [flag, str(x)]
        elif isinstance(v, bool):
            out += [flag, "true" if v else "false"]
        else:
            out += [flag, str(v)]
    return out


def _free_port(host):
    s = socket.socket()
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    s.bind((host, 0))
    port = s.getsockname()[1]
    s.close()
    return port


def supervise(a):
    from ..storage.remote import StoreServer
    store = StoreServer(wal=a.etcd_wal, fan_threads=a.etcd_fan_threads or None)
    addr = store.start()
    port = a.port or _free_port(a.bind_address)
    base = [sys.executable, "-m", "kubernetes_amd.cmd.apiserver", "--bind-address", a.bind_address,
            "--port", str(port), "--reuse-port", "--etcd-servers", addr,
            "-v", str(a.v)] + passthrough_args(a)
    ready_dir = store.dir or os.path.dirname(store.socket_path)
    children = []
    stopping = []

    def _stop(*_):
        stopping.append(1)
    signal.signal(signal.SIGTERM, _stop)
    signal.signal(signal.SIGINT, _stop)
    rc = 0
    try:
        for i in range(a.workers):
            pf = os.path.join(ready_dir, f"worker{i}.port")
            extra = []
            if a.audit_log_path:   # one audit file per worker process (no interleaved writes)
                extra += ["--audit-log-path", a.audit_log_path if a.audit_log_path == "-" else f"{a.audit_log_path}.w{i}"]
                if a.audit_policy_file:
                    extra += ["--audit-policy-file", a.audit_policy_file]
            children.append((subprocess.Popen(base + extra + ["--port-file", pf]), pf))
        t0 = time.time()
        while not all(os.path.exists(pf) for _, pf in children):
            if any(p.poll() is not None for p, _ in children) or time.time() - t0 > 120 or stopping:
                raise RuntimeError("API server workers failed to start")
            time.sleep(0.02)
        write_port_file(a.port_file, port)
        print(f"kube-apiserver: {a.workers} workers on http://{a.bind_address}:{port}, store {addr}", flush=True)
        while not stopping:
            dead = [p for p, _ in children if p.poll() is not None]
            if dead or store.proc.poll() is not None:
                print("kube-apiserver: a worker or the store exited; shutting down", file=sys.stderr, flush=True)
                rc = 1
                break
            time.sleep(0.2)
    finally:
        for p, _ in children:
            if p.poll() is None:
                p.terminate()
        for p, _ in children:
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                p.kill()
        store.stop()
    return rc


def _duration(v):
    from ..kubelet.kubeletconfig import parse_duration
    return parse_duration(v)


def _bool(v):
    return str(v).lower() not in ("false", "0", "no")


def _csv(v):
    return [x.strip() for x in (v or "").split(",") if x.strip()]


def _reference_flags(ap):
    """The rest of kube-apiserver's flags (cmd/kube-apiserver/app/options, generic server and
    kubeapiserver options). Flags for subsystems that do not exist here are accepted and marked."""
    g = ap.add_argument_group("serving")
    g.add_argument("--secure-port", type=int, default=0,
                   help="TLS listener with authentication (0 = single-listener mode on --port; the reference defaults to 6443)")
    g.add_argument("--insecure-port", dest="port", type=int, help="alias of --port (the insecure listener)")
    g.add_argument("--insecure-bind-address", "--address", dest="insecure_bind_address", default="127.0.0.1")
    g.add_argument("--cert-dir", default="/var/run/kubernetes", help="self-signed serving pair when --tls-cert-file is unset")
    g.add_argument("--advertise-address", default=None, help="IP published in the kubernetes service endpoints")
    g.add_argument("--apiserver-count", type=int, default=1)
    g.add_argument("--endpoint-reconciler-type", default="master-count", choices=["master-count", "lease", "none"])
    g.add_argument("--kubernetes-service-node-port", type=int, default=0)
    g.add_argument("--cors-allowed-origins", default="", help="comma-separated origin regular expressions")
    g.add_argument("--request-timeout", default="1m", help="non-long-running requests answer 504 after this ('0' = off)")
    g.add_argument("--min-request-timeout", type=int, default=1800,
                   help="watches without timeoutSeconds end after a random time in [t, 2t)")
    g.add_argument("--enable-logs-handler", type=_bool, default=True, help="/logs serves the API server's /var/log")
    g.add_argument("--enable-swagger-ui", type=_bool, default=False)
    g.add_argument("--profiling", type=_bool, default=True)
    g.add_argument("--runtime-config", default="", help="api/all=false, <group>/<version>=true|false, ...")
    g.add_argument("--allow-privileged", type=_bool, default=False)
    g = ap.add_argument_group("authentication / authorization")
    g.add_argument("--basic-auth-file", default=None)
    g.add_argument("--requestheader-client-ca-file", default=None)
    g.add_argument("--requestheader-allowed-names", default="")
    g.add_argument("--requestheader-username-headers", default="")
    g.add_argument("--requestheader-group-headers", default="")
    g.add_argument("--requestheader-extra-headers-prefix", default="")
    g.add_argument("--proxy-client-cert-file", default=None, help="client certificate for aggregated API servers")
    g.add_argument("--proxy-client-key-file", default=None)
    g.add_argument("--authentication-token-webhook-config-file", default=None, help="kubeconfig of the TokenReview webhook")
    g.add_argument("--authentication-token-webhook-cache-ttl", default="2m")
    g.add_argument("--authorization-webhook-config-file", default=None, help="kubeconfig of the SubjectAccessReview webhook")
    g.add_argument("--authorization-webhook-cache-authorized-ttl", default="5m")
    g.add_argument("--authorization-webhook-cache-unauthorized-ttl", default="30s")
    g.add_argument("--authorization-rbac-super-user", default=None)
    g = ap.add_argument_group("kubelet connections")
    g.add_argument("--kubelet-preferred-address-types", default="InternalIP,ExternalIP,Hostname,InternalDNS,ExternalDNS")
    g.add_argument("--kubelet-port", type=int, default=10250)
    deprecated_noop(g, "--kubelet-read-only-port", 10255, int, "options.go:202-203, 'DEPRECATED: kubelet port.'")
    g.add_argument("--kubelet-timeout", default="5s")
    g = ap.add_argument_group("audit")
    g.add_argument("--audit-log-format", default="json", choices=["json", "legacy"])
    g.add_argument("--audit-log-maxsize", type=int, default=0, help="MB before the audit log rotates")
    g.add_argument("--audit-log-maxbackup", type=int, default=0)
    g.add_argument("--audit-log-maxage", type=int, default=0, help="days a rotated audit log is kept")
    g.add_argument("--audit-webhook-mode", default="batch", choices=["batch", "blocking"],
                   help="batch: buffered, sent from a background thread; blocking: each request waits for its event")
    g.add_argument("--audit-webhook-batch-buffer-size", type=int, default=10000, help="events buffered before dropping")
    g.add_argument("--audit-webhook-batch-throttle-qps", type=float, default=10.0, help="batches per second (0 = off)")
    g.add_argument("--audit-webhook-batch-throttle-burst", type=int, default=15, help="batch burst above the qps")
    g.add_argument("--audit-webhook-batch-initial-backoff", default="10s", help="first retry delay of a failed batch")
    g = ap.add_argument_group("storage")
    g.add_argument("--storage-backend", default="etcd3", choices=["etcd3"])
    g.add_argument("--etcd-prefix", default="/registry",
                   help="key prefix in etcd: anything but /registry puts the keys under that namespace "
                        "(etcd v3 endpoints only)")
    g.add_argument("--etcd-compaction-interval", default="5m",
                   help="compact the store's history to the revision of one interval ago, every interval (0 = never)")
    unsupported(g, "--watch-cache", True, _bool, "every resource is served from its watch cache")
    g.add_argument("--watch-cache-sizes", default="",
                   help="per-resource watch windows, resource#size,... (e.g. pods#5000,nodes#1000)")
    g.add_argument("--default-watch-cache-size", type=int, default=None, help="alias of --watch-cache-size")
    unsupported(g, "--storage-versions", "", str, "each kind is stored in the version of its reference protobuf "
                "message (JSON for kinds outside the schema)")
    unsupported(g, "--storage-version", "", str, "see --storage-versions")
    unsupported(g, "--etcd-servers-overrides", "", str, "one store serves every resource")
    g.add_argument("--etcd-cafile", default="", help="CA of an https etcd endpoint")
    g.add_argument("--etcd-certfile", default="", help="client certificate for an https etcd endpoint")
    g.add_argument("--etcd-keyfile", default="", help="client key for an https etcd endpoint")
    unsupported(g, "--etcd-quorum-read", True, _bool, "every read is linearizable")
    unsupported(g, "--deserialization-cache-size", 0, int, "objects are decoded once into the watch cache")
    g.add_argument("--delete-collection-workers", type=int, default=1, help="concurrent deletes per DELETE-collection call")
    g.add_argument("--target-ram-mb", type=int, default=0,
                   help="size the watch windows for ~target/60 nodes (cachesize.go heuristics); "
                        "--watch-cache-sizes entries win")
    g = ap.add_argument_group("subsystems this API server does not have")
    g.add_argument("--cloud-provider", default="", help="'' only: cloud providers are out of scope")
    for f, why in (("--cloud-config", "cloud providers are out of scope"),
                   ("--external-hostname", "no cloud-derived external address; set --advertise-address"),
                   ("--experimental-keystone-url", "Keystone authentication is not implemented"),
                   ("--experimental-keystone-ca-file", "Keystone authentication is not implemented"),
                   ("--tls-ca-file", "the serving chain comes from --tls-cert-file"),
                   ("--tls-sni-cert-key", "one serving certificate (no SNI selection)"),
                   ("--kubeconfig", "kube-apiserver is not an aggregated API server"),
                   ("--authentication-kubeconfig", "kube-apiserver is not an aggregated API server"),
                   ("--authorization-kubeconfig", "kube-apiserver is not an aggregated API server")):
        unsupported(g, f, "", str, why)
    g.add_argument("--public-address-override", default="", help="deprecated alias of --bind-address")
    deprecated_noop(g, "--ssh-user", "", str, "options.go:159, SSH tunnels")
    deprecated_noop(g, "--ssh-keyfile", "", str, "options.go:164, SSH tunnels")
    unsupported(g, "--master-service-namespace", "default", str, "the kubernetes service lives in 'default'")
    unsupported(g, "--max-connection-bytes-per-sec", 0, int, "no per-connection rate limit")
    unsupported(g, "--http2-max-streams-per-connection", 0, int, "the server speaks HTTP/1.1")
    unsupported(g, "--enable-garbage-collector", True, _bool, "ownerReferences are always honoured")
    unsupported(g, "--enable-aggregator-routing", False, _bool, "aggregated APIs are reached through their service")
    unsupported(g, "--repair-malformed-updates", True, _bool, "updates are always defaulted from the stored object")
    unsupported(g, "--authentication-skip-lookup", False, _bool, "kube-apiserver is not an aggregated API server")
    g.add_argument("--contention-profiling", type=_bool, default=False,
                   help="sample where the event loop blocks, served at /debug/pprof/block (with --profiling)")


# `pkg/registry/cachesize/cachesize.go:25-44` NewHeuristicWatchCacheSizes: ~60 MB per node
_HEURISTIC = {"replicationcontrollers": (5, 100), "endpoints": (10, 1000), "nodes": (5, 1000),
              "pods": (50, 1000), "services": (5, 1000), "apiservices": (5, 1000)}


def watch_cache_sizes(target_ram_mb, spec):
    """--target-ram-mb heuristics, then --watch-cache-sizes `resource#size` entries on top
    (`ParseWatchCacheSizes`); plural -> window size."""
    sizes = {}
    if target_ram_mb and target_ram_mb > 0:
        cluster = target_ram_mb // 60
        sizes = {r: max(k * cluster, floor) for r, (k, floor) in _HEURISTIC.items()}
    for item in (x.strip() for x in (spec or "").split(",")):
        if not item:
            continue
        res, sep, n = item.partition("#")
        if not sep or not n.strip().lstrip("-").isdigit():
            raise ValueError(f"invalid --watch-cache-sizes entry {item!r} (want resource#size)")
        if int(n) <= 0:
            raise ValueError(f"--watch-cache-sizes {item!r}: the size must be positive "
                             "(every resource is served from its watch cache here)")
        sizes[res.strip().split(".", 1)[0]] = int(n)
    return sizes


def _reference_kwargs(a):
    if a.cloud_provider:
        raise SystemExit(f"kube-apiserver: --cloud-provider={a.cloud_provider}: cloud providers are out of scope here")
    from ..storage.etcd3_client import is_etcd3_address
    etcd3 = is_etcd3_address(a.etcd_servers or "")
    if a.etcd_prefix.rstrip("/") != "/registry" and not etcd3:
        raise SystemExit("kube-apiserver: --etcd-prefix other than /registry needs an etcd v3 endpoint in --etcd-servers")
    if (a.etcd_cafile or a.etcd_certfile or a.etcd_keyfile) and not etcd3:
        raise SystemExit("kube-apiserver: the kamd-etcd protocol has no TLS; reach the store over a unix socket "
                         "or a loopback/cluster-private TCP port (TLS flags apply to https etcd endpoints)")
    rh = None
    if a.requestheader_client_ca_file:
        rh = {"client_ca_file": a.requestheader_client_ca_file, "allowed_names": _csv(a.requestheader_allowed_names),
              "username_headers": _csv(a.requestheader_username_headers) or ["X-Remote-User"],
              "group_headers": _csv(a.requestheader_group_headers) or ["X-Remote-Group"],
              "extra_headers_prefix": _csv(a.requestheader_extra_headers_prefix) or ["X-Remote-Extra-"]}
    rt = _duration(a.request_timeout) if a.request_timeout not in ("0", "0s", "") else None
    return dict(basic_auth_file=a.basic_auth_file, requestheader=rh,
                authentication_token_webhook_config_file=a.authentication_token_webhook_config_file,
                authentication_token_webhook_cache_ttl=_duration(a.authentication_token_webhook_cache_ttl),
                authorization_webhook_config_file=a.authorization_webhook_config_file,
                authorization_webhook_cache_authorized_ttl=_duration(a.authorization_webhook_cache_authorized_ttl),
                authorization_webhook_cache_unauthorized_ttl=_duration(a.authorization_webhook_cache_unauthorized_ttl),
                authorization_rbac_super_user=a.authorization_rbac_super_user,
                cors_allowed_origins=_csv(a.cors_allowed_origins), request_timeout=rt,
                min_request_timeout=float(a.min_request_timeout), enable_logs_handler=a.enable_logs_handler,
                enable_swagger_ui=a.enable_swagger_ui, runtime_config=a.runtime_config or None,
                allow_privileged=a.allow_privileged,
                kubelet_preferred_address_types=_csv(a.kubelet_preferred_address_types),
                kubelet_port=a.kubelet_port, kubelet_timeout=_duration(a.kubelet_timeout),
                advertise_address=a.advertise_address, apiserver_count=a.apiserver_count,
                endpoint_reconciler_type=a.endpoint_reconciler_type,
                kubernetes_service_node_port=a.kubernetes_service_node_port,
                proxy_client_cert=(a.proxy_client_cert_file, a.proxy_client_key_file or a.proxy_client_cert_file)
                if a.proxy_client_cert_file else None,
                watch_cache_sizes=getattr(a, "watch_cache_sizes_map", None),
                compaction_interval=_duration(a.etcd_compaction_interval),
                delete_collection_workers=a.delete_collection_workers)


def main(argv=None):
    ap = _parser()
    a = ap.parse_args(argv)
    from ..utils.features import DefaultFeatureGate
    DefaultFeatureGate.set(a.feature_gates)
    check_unsupported(ap, a)
    if a.public_address_override:
        a.bind_address = a.public_address_override
    try:
        a.watch_cache_sizes_map = watch_cache_sizes(a.target_ram_mb, a.watch_cache_sizes)
    except ValueError as e:
        ap.error(str(e))
    setup_logging(a.v)
    if a.workers > 1 and not a.etcd_servers:
        sys.exit(supervise(a))

    async def start():
        store = a.etcd_servers
        etcd_tls = None
        from ..storage.etcd3_client import is_etcd3_address
        if store and is_etcd3_address(store):
            if a.etcd_prefix.rstrip("/") != "/registry":
                store = store.split("#", 1)[0] + "#" + a.etcd_prefix.rstrip("/")
            if a.etcd_cafile or a.etcd_certfile or a.etcd_keyfile:
                etcd_tls = (a.etcd_cafile or None, a.etcd_certfile or None, a.etcd_keyfile or None)
        if store is None and a.storage_engine == "native":
            try:
                from ..storage.native_store import NativeMVCCStore
                store = NativeMVCCStore(wal_path=a.etcd_wal)
            except (ImportError, OSError):
                store = None
        if store is None:
            store = MVCCStore(wal_path=a.etcd_wal)
        plugins = a.admission_control.split(",") if a.admission_control else None
        adm_cfg = load_admission_config(a.admission_control_config_file) if a.admission_control_config_file else None
        audit = None
        if a.audit_log_path or a.audit_webhook_config_file:
            from ..apiserver.audit import AuditLogger, Policy, WebhookBackend
            wh = (WebhookBackend(a.audit_webhook_config_file, a.audit_webhook_batch_max_size, a.audit_webhook_batch_max_wait,
                                 buffer=a.audit_webhook_batch_buffer_size, mode=a.audit_webhook_mode,
                                 throttle_qps=a.audit_webhook_batch_throttle_qps,
                                 throttle_burst=a.audit_webhook_batch_throttle_burst,
                                 initial_backoff=_duration(a.audit_webhook_batch_initial_backoff))
                  if a.audit_webhook_config_file else None)
            audit = AuditLogger(a.audit_log_path, Policy.load(a.audit_policy_file) if a.audit_policy_file else None,
                                webhook=wh, format=a.audit_log_format, max_size_mb=a.audit_log_maxsize,
                                max_backups=a.audit_log_maxbackup, max_age_days=a.audit_log_maxage)
        oidc = None
        if a.oidc_issuer_url:
            oidc = {"issuer_url": a.oidc_issuer_url, "client_id": a.oidc_client_id,
                    "username_claim": a.oidc_username_claim, "username_prefix": a.oidc_username_prefix,
                    "groups_claim": a.oidc_groups_claim, "groups_prefix": a.oidc_groups_prefix, "ca_file": a.oidc_ca_file,
                    "required_claims": dict(x.split("=", 1) for x in a.oidc_required_claim)}
        s = APIServer(store=store, etcd_tls=etcd_tls, admission_plugins=plugins, admission_config=adm_cfg, token_file=a.token_auth_file,
                      authorization_modes=a.authorization_mode.split(","), storage_media_type=a.storage_media_type,
                      max_requests_inflight=a.max_requests_inflight,
                      max_mutating_inflight=a.max_mutating_requests_inflight, watch_window=a.default_watch_cache_size or a.watch_cache_size,
                      event_ttl=_duration(a.event_ttl),
                      audit=audit, encryption_config=a.encryption_config,
                      service_cluster_ip_range=a.service_cluster_ip_range,
                      service_node_port_range=tuple(int(x) for x in a.service_node_port_range.split("-")),
                      kubelet_https=a.kubelet_https, kubelet_certificate_authority=a.kubelet_certificate_authority,
                      kubelet_client_certificate=a.kubelet_client_certificate, kubelet_client_key=a.kubelet_client_key,
                      tls_cert_file=a.tls_cert_file, tls_private_key_file=a.tls_private_key_file,
                      client_ca_file=a.client_ca_file, service_account_key_files=a.service_account_key_file,
                      service_account_lookup=a.service_account_lookup,
                      enable_bootstrap_token_auth=a.enable_bootstrap_token_auth,
                      authentication_token_webhook=a.authentication_token_webhook_url, anonymous_auth=a.anonymous_auth,
                      authorization_policy_file=a.authorization_policy_file,
                      authorization_webhook_url=a.authorization_webhook_url, oidc=oidc, **_reference_kwargs(a))
        s.enable_profiling = a.profiling
        if a.contention_profiling and a.profiling:
            from ..utils.profiling import enable_contention_profiling
            enable_contention_profiling()
        if a.secure_port:
            # the reference's two listeners: TLS + authn/authz on --bind-address:--secure-port
            # (self-signed in --cert-dir without --tls-cert-file), plain HTTP without either on
            # --insecure-bind-address:--port/--insecure-port (0 = off)
            if not a.tls_cert_file:
                from ..utils.tlsutil import self_signed_serving_cert
                cert, key = self_signed_serving_cert(a.cert_dir, "kube-apiserver",
                                                     [a.advertise_address, "kubernetes", "kubernetes.default",
                                                      "kubernetes.default.svc"], basename="apiserver")
                s.tls = (cert, key, a.client_ca_file)
            sport = await s.start(a.bind_address, a.secure_port, reuse_port=a.reuse_port)
            iport = await s.start_insecure(a.insecure_bind_address, a.port, reuse_port=a.reuse_port) if a.port else None
            write_port_file(a.port_file, iport or sport)
            if not a.reuse_port:
                print(f"kube-apiserver listening on https://{a.bind_address}:{sport}"
                      + (f" and http://{a.insecure_bind_address}:{iport} (insecure)" if iport else ""), flush=True)
            return s
        port = await s.start(a.bind_address, a.port, reuse_port=a.reuse_port)
        write_port_file(a.port_file, port)
        if not a.reuse_port:
            print(f"kube-apiserver listening on http{'s' if a.tls_cert_file else ''}://{a.bind_address}:{port}", flush=True)
        return s

    run_until_signal(start)


if __name__ == "__main__":
    main()
