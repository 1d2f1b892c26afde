"""`kubeadm` command line: init, join, token, reset, upgrade, config, phase, version.

Parity: `cmd/kubeadm/app/cmd/{init,join,token,reset,config,version}.go`, `cmd/upgrade/*` and `cmd/phases/*` (each
init phase is runnable on its own as `kubeadm phase <name>`).
"""
from __future__ import annotations

import argparse
import asyncio
import os
import subprocess
import sys
import time

import yaml

from ..client import clientcmd
from ..client.rest import APIStatusError
from . import phases as P


def _cfg_from(a):
    cfg = P.default_config()
    if getattr(a, "config", None):
        with open(a.config) as f:
            cfg = P.default_config(**(yaml.safe_load(f) or {}))
    over = {}
    if getattr(a, "apiserver_advertise_address", None):
        over.setdefault("api", {})["advertiseAddress"] = a.apiserver_advertise_address
    if getattr(a, "apiserver_bind_port", None):
        over.setdefault("api", {})["bindPort"] = a.apiserver_bind_port
    if getattr(a, "service_cidr", None):
        over.setdefault("networking", {})["serviceSubnet"] = a.service_cidr
    if getattr(a, "pod_network_cidr", None):
        over.setdefault("networking", {})["podSubnet"] = a.pod_network_cidr
    for k, attr in (("nodeName", "node_name"), ("token", "token"), ("tokenTTL", "token_ttl"),
                    ("certificatesDir", "cert_dir"), ("kubernetesDir", "kubernetes_dir")):
        if getattr(a, attr, None):
            over[k] = getattr(a, attr)
    for k, v in over.items():
        if isinstance(v, dict):
            cfg[k].update(v)
        else:
            cfg[k] = v
    if getattr(a, "kubernetes_dir", None) and not getattr(a, "cert_dir", None) and not getattr(a, "config", None):
        cfg["certificatesDir"] = os.path.join(cfg["kubernetesDir"], "pki")
    return cfg


async def _wait_api(client, timeout):
    end = time.monotonic() + timeout
    last = None
    while time.monotonic() < end:
        try:
            await client.get("namespaces", "kube-system")
            return
        except Exception as e:  # noqa: BLE001 - apiserver not up yet
            last = e
            await asyncio.sleep(0.5)
    raise TimeoutError(f"the control plane did not become healthy within {timeout}s: {last}")


async def _wait_node(client, name, timeout):
    end = time.monotonic() + timeout
    while time.monotonic() < end:
        try:
            return await client.get("nodes", name)
        except APIStatusError as e:
            if e.code != 404:
                raise
        await asyncio.sleep(0.5)
    raise TimeoutError(f"node {name} did not register within {timeout}s")


async def post_control_plane(cfg, admin_kubeconfig, token, wait_timeout=300.0, mark_master=True, out=print):
    """The init phases that need a running API server."""
    client = clientcmd.client_from(admin_kubeconfig)
    try:
        await _wait_api(client, wait_timeout)
        out("[apiclient] control plane is healthy")
        await P.phase_upload_config(client, cfg)
        out("[uploadconfig] stored MasterConfiguration in ConfigMap kube-system/kubeadm-config")
        if mark_master:
            await _wait_node(client, cfg["nodeName"], wait_timeout)
            await P.phase_mark_master(client, cfg["nodeName"])
            out(f"[markmaster] labelled and tainted {cfg['nodeName']} as master")
        await P.phase_bootstrap_token(client, cfg, token)
        out(f"[bootstraptoken] using token: {token}")
        await P.phase_cluster_info(client, cfg)
        out("[bootstraptoken] created cluster-info ConfigMap in kube-public")
        await P.phase_addons(client, cfg)
        out("[addons] applied kube-proxy and amd-gpu-device-plugin")
    finally:
        await client.close()


def _join_command(cfg, token):
    ca = open(os.path.join(cfg["certificatesDir"], "ca.crt")).read()
    return (f"kubeadm join --token {token} {cfg['api']['advertiseAddress']}:{cfg['api']['bindPort']} "
            f"--discovery-token-ca-cert-hash {P.ca_cert_hash(ca)}")


def cmd_init(a):
    cfg = _cfg_from(a)
    token = cfg.get("token") or P.generate_token()
    if not a.skip_preflight_checks:
        warns, errs = P.preflight(cfg)
        for w in warns:
            print(f"[preflight] WARNING: {w}")
        if errs:
            for e in errs:
                print(f"[preflight] ERROR: {e}", file=sys.stderr)
            return 1
    made = P.phase_certs(cfg)
    print(f"[certificates] generated {', '.join(made) or 'nothing (all present)'} in {cfg['certificatesDir']}")
    print(f"[kubeconfig] wrote {', '.join(P.phase_kubeconfig(cfg)) or 'nothing (all present)'} to {cfg['kubernetesDir']}")
    for p in P.phase_manifests(cfg):
        print(f"[controlplane] wrote static pod manifest {p}")
    if a.dry_run:
        return 0
    if a.start_kubelet:
        kd = cfg["kubernetesDir"]
        log = open(os.path.join(kd, "kubelet.log"), "ab")
        subprocess.Popen([sys.executable, "-m", "kubernetes_amd.cmd.kubelet", "--kubeconfig", os.path.join(kd, P.KUBELET_CONF),
                          "--pod-manifest-path", os.path.join(kd, "manifests"), "--hostname-override", cfg["nodeName"],
                          "--root-dir", os.path.join(kd, "kubelet")] + P.kubelet_flags(cfg["certificatesDir"]),
                         stdout=log, stderr=log, start_new_session=True)
        print("[kubelet] started kubelet (static pods will bring up the control plane)")
    asyncio.run(post_control_plane(cfg, os.path.join(cfg["kubernetesDir"], P.ADMIN_CONF), token, a.timeout,
                                   mark_master=not a.skip_mark_master))
    print("\nYour Kubernetes master has initialized successfully!\n\nTo start using your cluster:\n"
          f"  mkdir -p $HOME/.kube && cp {os.path.join(cfg['kubernetesDir'], P.ADMIN_CONF)} $HOME/.kube/config\n\n"
          "Join MI355X nodes by running on each as root:\n\n  " + _join_command(cfg, token))
    return 0


def cmd_join(a):
    server = a.server if a.server.startswith("http") else f"https://{a.server}"
    token = a.discovery_token or a.token
    if not token:
        print("join: --token or --discovery-token is required", file=sys.stderr)
        return 1
    node = a.node_name or P.default_config()["nodeName"]
    conf = asyncio.run(P.join(server, token, node, a.kubernetes_dir, tuple(a.discovery_token_ca_cert_hash or ()),
                              a.discovery_token_unsafe_skip_ca_verification, a.timeout))
    print(f"[join] TLS bootstrap complete, kubelet credentials in {conf}\n\nThis node has joined the cluster.")
    if a.start_kubelet:
        subprocess.Popen([sys.executable, "-m", "kubernetes_amd.cmd.kubelet", "--kubeconfig", conf,
                          "--hostname-override", node, "--root-dir", os.path.join(a.kubernetes_dir, "kubelet")]
                         + P.kubelet_flags(os.path.join(a.kubernetes_dir, "pki")), start_new_session=True)
    return 0


async def _tokens(a, op):
    client = clientcmd.client_from(a.kubeconfig)
    try:
        if op == "create":
            tok = a.token or P.generate_token()
            usages = [u.strip() for u in a.usages.split(",") if u.strip()]
            groups = [g.strip() for g in a.groups.split(",") if g.strip()]
            await client.create("secrets", P.token_secret(tok, P.parse_ttl(a.ttl), usages, groups, a.description),
                                "kube-system")
            print(tok)
            if a.print_join_command:
                cfg = P.default_config(certificatesDir=a.cert_dir or "/etc/kubernetes/pki")
                kc, _ = clientcmd.load(a.kubeconfig)
                srv = kc["clusters"][0]["cluster"]["server"].split("://", 1)[-1]
                ca = open(os.path.join(cfg["certificatesDir"], "ca.crt")).read()
                print(f"kubeadm join --token {tok} {srv} --discovery-token-ca-cert-hash {P.ca_cert_hash(ca)}")
        elif op == "list":
            import base64
            lst = await client.list("secrets", "kube-system")
            print(f"{'TOKEN':<24}{'EXPIRES':<22}{'USAGES':<28}{'EXTRA GROUPS'}")
            for s in lst["items"]:
                if s.get("type") != "bootstrap.kubernetes.io/token":
                    continue
                d = {k: base64.b64decode(v).decode() for k, v in (s.get("data") or {}).items()}
                usages = ",".join(sorted(k[len("usage-bootstrap-"):] for k, v in d.items()
                                         if k.startswith("usage-bootstrap-") and v == "true"))
                print(f"{d.get('token-id', '')}.{d.get('token-secret', ''):<{24 - len(d.get('token-id', '')) - 1}}"
                      f"{d.get('expiration', '<forever>'):<22}{usages:<28}{d.get('auth-extra-groups', '')}")
        elif op == "delete":
            tid = a.token_value.split(".")[0]
            await client.delete("secrets", f"bootstrap-token-{tid}", "kube-system")
            print(f"bootstrap token with id {tid!r} deleted")
    finally:
        await client.close()
    return 0


def cmd_phase(a):
    cfg = _cfg_from(a)
    if a.phase == "preflight":
        w, e = P.preflight(cfg)
        print("\n".join([f"WARNING: {x}" for x in w] + [f"ERROR: {x}" for x in e]) or "preflight checks passed")
        return 1 if e else 0
    if a.phase == "certs":
        print("\n".join(P.phase_certs(cfg)))
    elif a.phase == "kubeconfig":
        print("\n".join(P.phase_kubeconfig(cfg)))
    elif a.phase == "controlplane":
        print("\n".join(p for p in P.phase_manifests(cfg) if not p.endswith("/etcd.yaml")))
    elif a.phase == "etcd":
        if cfg["etcd"].get("endpoints"):
            print("external store configured (etcd.endpoints): no local etcd manifest")
        else:
            print(P.phase_etcd_local(cfg))
    else:
        admin = os.path.join(cfg["kubernetesDir"], P.ADMIN_CONF)

        async def go():
            c = clientcmd.client_from(admin)
            try:
                if a.phase == "upload-config":
                    await P.phase_upload_config(c, cfg)
                elif a.phase == "mark-master":
                    await P.phase_mark_master(c, cfg["nodeName"])
                elif a.phase == "bootstrap-token":
                    tok = cfg.get("token") or P.generate_token()
                    await P.phase_bootstrap_token(c, cfg, tok)
                    await P.phase_cluster_info(c, cfg)
                    print(tok)
                elif a.phase == "addons":
                    await P.phase_addons(c, cfg)
            finally:
                await c.close()
        asyncio.run(go())
    return 0


def cmd_upgrade(a):
    """`kubeadm upgrade plan|apply` (kubeadm/upgrade.py)."""
    from . import upgrade as U

    def confirm():
        if a.yes:
            return True
        ans = input("[upgrade/confirm] Are you sure you want to proceed with the upgrade? [y/N]: ")
        return ans.strip().lower() in ("y", "yes")

    async def go():
        c = clientcmd.client_from(a.kubeconfig)
        try:
            cfg = await U.fetch_config(c, a.config)
            if a.op == "plan":
                if not a.skip_preflight_checks:
                    errs = await U.health_checks(c, cfg)
                    if errs:
                        raise U.UpgradeError("[upgrade/health] FATAL: " + "; ".join(errs))
                await U.plan(c, cfg)
            else:
                await U.apply(c, cfg, a.version, force=a.force, dry_run=a.dry_run,
                              allow_experimental=a.allow_experimental_upgrades,
                              allow_rc=a.allow_release_candidate_upgrades, skip_preflight=a.skip_preflight_checks,
                              timeout=a.timeout, confirm=confirm)
        finally:
            await c.close()
    try:
        asyncio.run(go())
    except U.UpgradeError as e:
        print(str(e), file=sys.stderr)
        return 1
    return 0


def _common(p):
    p.add_argument("--config", default=None, help="MasterConfiguration YAML")
    p.add_argument("--kubernetes-dir", default=None)
    p.add_argument("--cert-dir", default=None)
    p.add_argument("--node-name", default=None)
    p.add_argument("--apiserver-advertise-address", default=None)
    p.add_argument("--apiserver-bind-port", type=int, default=None)
    p.add_argument("--service-cidr", default=None)
    p.add_argument("--pod-network-cidr", default=None)
    p.add_argument("--token", default=None)
    p.add_argument("--token-ttl", default=None)


def main(argv=None):
    ap = argparse.ArgumentParser(prog="kubeadm")
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("init")
    _common(p)
    p.add_argument("--skip-preflight-checks", action="store_true")
    p.add_argument("--skip-mark-master", action="store_true")
    p.add_argument("--dry-run", action="store_true", help="write certs/kubeconfigs/manifests only")
    p.add_argument("--start-kubelet", action="store_true", help="launch the kubelet on the static pod manifests")
    p.add_argument("--timeout", type=float, default=300.0)
    p = sub.add_parser("join")
    p.add_argument("server", help="API server host:port")
    p.add_argument("--token", default=None)
    p.add_argument("--discovery-token", default=None)
    p.add_argument("--discovery-token-ca-cert-hash", action="append", default=[])
    p.add_argument("--discovery-token-unsafe-skip-ca-verification", action="store_true")
    p.add_argument("--node-name", default=None)
    p.add_argument("--kubernetes-dir", default="/etc/kubernetes")
    p.add_argument("--start-kubelet", action="store_true")
    p.add_argument("--timeout", type=float, default=300.0)
    p = sub.add_parser("token")
    tsub = p.add_subparsers(dest="op", required=True)
    for op in ("create", "list", "delete"):
        q = tsub.add_parser(op)
        q.add_argument("--kubeconfig", default="/etc/kubernetes/admin.conf")
        if op == "create":
            q.add_argument("token", nargs="?", default=None)
            q.add_argument("--ttl", default="24h")
            q.add_argument("--usages", default="signing,authentication")
            q.add_argument("--groups", default=P.BOOTSTRAP_GROUP)
            q.add_argument("--description", default="")
            q.add_argument("--print-join-command", action="store_true")
            q.add_argument("--cert-dir", default=None)
        if op == "delete":
            q.add_argument("token_value")
    tsub.add_parser("generate")
    p = sub.add_parser("reset")
    _common(p)
    p = sub.add_parser("phase")
    p.add_argument("phase", choices=["preflight", "certs", "kubeconfig", "etcd", "controlplane", "upload-config",
                                     "mark-master", "bootstrap-token", "addons"])
    _common(p)
    p = sub.add_parser("upgrade")
    usub = p.add_subparsers(dest="op", required=True)
    for op in ("plan", "apply"):
        q = usub.add_parser(op)
        if op == "apply":
            q.add_argument("version")
            q.add_argument("-f", "--force", action="store_true")
            q.add_argument("-y", "--yes", action="store_true")
            q.add_argument("--dry-run", action="store_true")
            q.add_argument("--timeout", type=float, default=300.0, help="seconds to wait for each static pod")
        q.add_argument("--config", default=None)
        q.add_argument("--kubeconfig", default="/etc/kubernetes/admin.conf")
        q.add_argument("--allow-experimental-upgrades", action="store_true")
        q.add_argument("--allow-release-candidate-upgrades", action="store_true")
        q.add_argument("--skip-preflight-checks", action="store_true")
    p = sub.add_parser("config")
    p.add_argument("op", choices=["view", "print-default"])
    p.add_argument("--kubeconfig", default="/etc/kubernetes/admin.conf")
    sub.add_parser("version")
    a = ap.parse_args(argv)
    if a.cmd == "init":
        return cmd_init(a)
    if a.cmd == "join":
        return cmd_join(a)
    if a.cmd == "token":
        if a.op == "generate":
            print(P.generate_token())
            return 0
        return asyncio.run(_tokens(a, a.op))
    if a.cmd == "reset":
        P.reset(_cfg_from(a))
        print("[reset] removed manifests, kubeconfigs, certificates and store data")
        return 0
    if a.cmd == "phase":
        return cmd_phase(a)
    if a.cmd == "upgrade":
        return cmd_upgrade(a)
    if a.cmd == "config":
        if a.op == "print-default":
            print(yaml.safe_dump(P.default_config(), sort_keys=False))
            return 0

        async def view():
            c = clientcmd.client_from(a.kubeconfig)
            try:
                cm = await c.get("configmaps", "kubeadm-config", "kube-system")
                print(cm["data"]["MasterConfiguration"])
            finally:
                await c.close()
        asyncio.run(view())
        return 0
    if a.cmd == "version":
        print(f"kubeadm version: {P.VERSION}")
    return 0
