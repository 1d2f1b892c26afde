"""`kubeadm upgrade plan|apply`: in-place control-plane upgrade of a kubeadm cluster.

Parity: `cmd/kubeadm/app/cmd/upgrade/{plan,apply,common}.go` and `cmd/kubeadm/app/phases/upgrade/`:

* the cluster's MasterConfiguration is read back from ConfigMap `kube-system/kubeadm-config`
  (or `--config`), the target version is written into it (`configuration.go`);
* health preflight (`health.go`): the API server answers /healthz, every node is Ready, and
  every control-plane static pod manifest exists;
* version-skew policy (`policy.go` EnforceVersionPolicies): at most one minor version up or
  down, nothing at/below the minimum control-plane version, not past kubeadm's own minor,
  kubelets at most one minor behind; unstable (alpha/beta/rc) targets need
  `--allow-experimental-upgrades` / `--allow-release-candidate-upgrades`. Mandatory errors
  always stop the upgrade; skippable ones only without `--force`. A `-amd.N` suffix is this
  distribution's build number, not a pre-release;
* static-pod upgrade (`staticpods.go`): new manifests are rendered into a temp dir, the store's
  data directory is backed up (it lives in the API server's static pod here, so this takes the
  place of the reference's etcd backup), then component by component the live manifest moves
  to the backup dir, the new one moves in, and kubeadm waits for the kubelet to restart the
  static pod (mirror pod `kubernetes.io/config.hash` changes) and for the pod to run again;
  any failure moves every backed-up manifest back (rollbackOldManifests);
* post-upgrade (`postupgrade.go`): the new configuration is uploaded, the bootstrap-token RBAC
  rules are re-applied and the kube-proxy / GPU device-plugin add-ons are updated to the new
  version;
* `plan` (`plan.go`): cluster, kubeadm and kubelet versions and what `apply` would do (there
  is no network here, so the candidate is kubeadm's own version rather than dl.k8s.io's
  stable.txt).
"""
from __future__ import annotations

import asyncio
import os
import re
import shutil
import tempfile
import time

import yaml

from ..client.rest import APIStatusError
from . import phases as P

MINIMUM_CONTROL_PLANE_VERSION = "v1.8.0"
MAX_UPGRADE_SKEW = MAX_DOWNGRADE_SKEW = MAX_KUBELET_SKEW = 1
COMPONENTS = ("kube-apiserver", "kube-controller-manager", "kube-scheduler")
CONFIG_HASH = "kubernetes.io/config.hash"

_VER = re.compile(r"^v?(\d+)\.(\d+)\.(\d+)(?:-([0-9A-Za-z.-]+))?(?:\+[0-9A-Za-z.-]+)?$")


class UpgradeError(Exception):
    pass


class Version:
    """Semantic version (`pkg/util/version`). `-amd.N` is a distribution build (stable, ordered
    by N); any other pre-release (alpha/beta/rc) sorts before the release."""

    def __init__(self, text: str):
        m = _VER.match(text.strip())
        if not m:
            raise ValueError(f"could not parse {text!r} as a version")
        self.text = text.strip()
        self.major, self.minor, self.patch = int(m.group(1)), int(m.group(2)), int(m.group(3))
        pre = m.group(4) or ""
        self.build = 0
        if pre.startswith("amd"):
            self.build = int(pre.split(".")[1]) if "." in pre and pre.split(".")[1].isdigit() else 0
            pre = ""
        self.pre = pre

    def _key(self):
        pre_ids = tuple((0, int(p), "") if p.isdigit() else (1, 0, p) for p in self.pre.split(".")) if self.pre else ()
        return (self.major, self.minor, self.patch, 0 if self.pre else 1, pre_ids, self.build)

    def __lt__(self, o):
        return self._key() < o._key()

    def __le__(self, o):
        return self._key() <= o._key()

    def __eq__(self, o):
        return isinstance(o, Version) and self._key() == o._key()

    def __hash__(self):
        return hash(self._key())

    def __str__(self):
        return self.text


def enforce_version_policies(new: str, cluster: str, kubeadm: str, kubelets: dict,
                             allow_experimental=False, allow_rc=False):
    """-> (mandatory errors, skippable errors)."""
    mandatory, skippable = [], []
    nv, cv, kv = Version(new), Version(cluster), Version(kubeadm)
    if nv <= Version(MINIMUM_CONTROL_PLANE_VERSION):
        mandatory.append(f"Specified version to upgrade to {new!r} is equal to or lower than the minimum supported "
                         f"version {MINIMUM_CONTROL_PLANE_VERSION!r}. Please specify a higher version to upgrade to")
    if nv.minor > cv.minor + MAX_UPGRADE_SKEW:
        (skippable if nv.pre else mandatory).append(
            f"Specified version to upgrade to {new!r} is too high; kubeadm can upgrade only {MAX_UPGRADE_SKEW} minor "
            "version at a time")
    if nv.minor < cv.minor - MAX_DOWNGRADE_SKEW:
        (skippable if nv.pre else mandatory).append(
            f"Specified version to downgrade to {new!r} is too low; kubeadm can downgrade only {MAX_DOWNGRADE_SKEW} "
            "minor version at a time")
    if kv < nv:
        if nv.minor > kv.minor:
            (skippable if nv.pre else mandatory).append(
                f"Specified version to upgrade to {new!r} is at least one minor release higher than the kubeadm minor "
                f"release ({nv.minor} > {kv.minor}). Such an upgrade is not supported")
        else:
            skippable.append(f"Specified version to upgrade to {new!r} is higher than the kubeadm version {kubeadm!r}. "
                             "Upgrade kubeadm first using the tool you used to install kubeadm")
    if nv.pre and not allow_experimental and not (nv.pre.startswith("rc") and allow_rc):
        skippable.append(f"Specified version to upgrade to {new!r} is an unstable version and such upgrades weren't "
                         "allowed via setting the --allow-*-upgrades flags")
    old = sorted(v for v in kubelets if nv.minor > Version(v).minor + MAX_KUBELET_SKEW)
    if old:
        skippable.append(f"There are kubelets in this cluster that are too old that have these versions {old}")
    return mandatory, skippable


# ------------------------------------------------------------------------------------ cluster state
async def fetch_config(client, config_path=None):
    if config_path:
        with open(config_path) as f:
            return P.default_config(**(yaml.safe_load(f) or {}))
    try:
        cm = await client.get("configmaps", "kubeadm-config", "kube-system")
    except APIStatusError as e:
        raise UpgradeError(f"could not read the kubeadm configuration from kube-system/kubeadm-config: {e}; "
                           "pass --config") from e
    return P.default_config(**(yaml.safe_load((cm.get("data") or {}).get("MasterConfiguration") or "") or {}))


async def versions(client):
    """(cluster version, kubeadm version, {kubelet version: node count})."""
    st, body = await client.raw("GET", "/version")
    if st != 200:
        raise UpgradeError(f"could not fetch the cluster version: HTTP {st}")
    cluster = yaml.safe_load(body)["gitVersion"]
    kubelets: dict[str, int] = {}
    for n in (await client.list("nodes"))["items"]:
        v = ((n.get("status") or {}).get("nodeInfo") or {}).get("kubeletVersion")
        if v:
            kubelets[v] = kubelets.get(v, 0) + 1
    return cluster, P.VERSION, kubelets


async def health_checks(client, cfg):
    """`health.go` CheckClusterHealth: -> list of failures."""
    errs = []
    st, _ = await client.raw("GET", "/healthz")
    if st != 200:
        errs.append(f"the API Server is unhealthy; /healthz didn't return \"ok\" (HTTP {st})")
    not_ready = []
    for n in (await client.list("nodes"))["items"]:
        ready = any(c.get("type") == "Ready" and c.get("status") == "True"
                    for c in (n.get("status") or {}).get("conditions") or ())
        if not ready:
            not_ready.append(n["metadata"]["name"])
    if not_ready:
        errs.append(f"there are NotReady Nodes in the cluster: {not_ready}")
    mdir = os.path.join(cfg["kubernetesDir"], "manifests")
    for comp in COMPONENTS:
        if not os.path.exists(os.path.join(mdir, comp + ".yaml")):
            errs.append(f"the static pod manifest for component {comp} doesn't exist in {mdir}")
    return errs


async def static_pod_hash(client, node, component):
    try:
        p = await client.get("pods", f"{component}-{node}", "kube-system")
    except (APIStatusError, OSError, ConnectionError):
        return None
    return ((p.get("metadata") or {}).get("annotations") or {}).get(CONFIG_HASH)


async def _wait(pred, timeout, what, interval=0.2):
    end = time.monotonic() + timeout
    while time.monotonic() < end:
        try:
            if await pred():
                return
        except (APIStatusError, OSError, ConnectionError, asyncio.TimeoutError):
            pass    # the API server itself may be restarting
        await asyncio.sleep(interval)
    raise UpgradeError(f"timed out waiting for {what}")


# ------------------------------------------------------------------------------------ apply
class StaticPodPaths:
    """Real / upgraded / backup manifest directories (`KubeStaticPodPathManager`)."""

    def __init__(self, real_dir, tmp_root=None):
        self.real = real_dir
        root = tmp_root or os.path.join(os.path.dirname(real_dir.rstrip("/")), "tmp")
        os.makedirs(root, exist_ok=True)
        self.new = tempfile.mkdtemp(prefix="kubeadm-upgraded-manifests", dir=root)
        self.backup = tempfile.mkdtemp(prefix="kubeadm-backup-manifests", dir=root)
        self.backup_store = tempfile.mkdtemp(prefix="kubeadm-backup-etcd", dir=root)

    def path(self, kind, comp):
        return os.path.join(getattr(self, kind), comp + ".yaml")


def rollback(paths: StaticPodPaths, recover: dict, out=print):
    for comp, backup in recover.items():
        if os.path.exists(backup):
            os.replace(backup, paths.path("real", comp))
            out(f"[upgrade/rollback] restored the manifest of {comp}")


async def upgrade_component(client, cfg, comp, paths, before_hash, recover, timeout, out=print):
    recover[comp] = paths.path("backup", comp)
    os.replace(paths.path("real", comp), paths.path("backup", comp))
    os.replace(paths.path("new", comp), paths.path("real", comp))
    out(f"[upgrade/staticpods] Moved new manifest to {paths.path('real', comp)!r} and backed up old manifest to "
        f"{paths.path('backup', comp)!r}")
    out("[upgrade/staticpods] Waiting for the kubelet to restart the component")
    node = cfg["nodeName"]

    async def hash_changed():
        h = await static_pod_hash(client, node, comp)
        return h is not None and h != before_hash

    async def running():
        pods = (await client.list("pods", "kube-system", label_selector=f"component={comp}"))["items"]
        return bool(pods) and all((p.get("status") or {}).get("phase") == "Running" for p in pods)
    await _wait(hash_changed, timeout, f"the static pod of {comp} to be restarted by the kubelet")
    await _wait(running, timeout, f"the pods with label component={comp} to run")
    out(f"[upgrade/staticpods] Component {comp!r} upgraded successfully!")


async def apply(client, cfg, new_version, *, force=False, dry_run=False, allow_experimental=False, allow_rc=False,
                skip_preflight=False, timeout=300.0, confirm=None, out=print):
    """The whole `kubeadm upgrade apply` flow; returns the upgraded configuration."""
    if not skip_preflight:
        errs = await health_checks(client, cfg)
        if errs:
            raise UpgradeError("[upgrade/health] FATAL: " + "; ".join(errs))
        out("[upgrade] Making sure the cluster is healthy: all nodes Ready, control-plane manifests present")
    cluster, kubeadm_v, kubelets = await versions(client)
    mandatory, skippable = enforce_version_policies(new_version, cluster, kubeadm_v, kubelets, allow_experimental, allow_rc)
    if mandatory:
        raise UpgradeError("[upgrade/version] FATAL: the --version argument is invalid due to these fatal errors:\n"
                           + "\n".join(f"\t- {e}" for e in mandatory))
    if skippable:
        if not force:
            raise UpgradeError("[upgrade/version] FATAL: the --version argument is invalid due to these errors:\n"
                               + "\n".join(f"\t- {e}" for e in skippable) + "\nCan be bypassed if you pass the --force flag")
        for e in skippable:
            out(f"[upgrade/version] Found {len(skippable)} potential version compatibility errors but skipping since the "
                f"--force flag is set: {e}")
    out(f"[upgrade/version] You have chosen to change the cluster version to {new_version!r}")
    new_cfg = dict(cfg, kubernetesVersion=new_version)
    manifests = P.control_plane_manifests(new_cfg)
    if dry_run:
        for comp in COMPONENTS:
            out(f"[dryrun] Would write file {os.path.join(cfg['kubernetesDir'], 'manifests', comp + '.yaml')} with content:")
            out(yaml.safe_dump(manifests[comp], sort_keys=False))
        out("[upgrade/successful] SUCCESS! (dry run: nothing was changed)")
        return new_cfg
    if confirm is not None and not confirm():
        raise UpgradeError("[upgrade/confirm] Upgrade aborted by the user")
    paths = StaticPodPaths(os.path.join(cfg["kubernetesDir"], "manifests"))
    for comp in COMPONENTS:
        P._write(paths.path("new", comp), yaml.safe_dump(manifests[comp], sort_keys=False))
    data = cfg.get("etcd", {}).get("dataDir")
    if data and os.path.isdir(data):
        shutil.copytree(data, os.path.join(paths.backup_store, "data"), dirs_exist_ok=True)
        out(f"[upgrade/staticpods] Backed up the store data to {paths.backup_store!r}")
    out(f"[upgrade/staticpods] Writing new Static Pod manifests to {paths.new!r}")
    recover: dict[str, str] = {}
    for comp in COMPONENTS:
        # the current hash must be known: a mirror pod caught mid-recreation (no hash yet) would
        # make ANY later hash look like a restart (`WaitForStaticPodHash` reads it first too)
        before = None
        end = time.monotonic() + min(timeout, 10.0)
        while before is None and time.monotonic() < end:
            before = await static_pod_hash(client, cfg["nodeName"], comp)
            if before is None:
                await asyncio.sleep(0.1)
        try:
            await upgrade_component(client, cfg, comp, paths, before, recover, timeout, out)
        except (UpgradeError, OSError) as e:
            rollback(paths, recover, out)
            raise UpgradeError(f"[upgrade/apply] FATAL: couldn't upgrade control plane. kubeadm has tried to recover "
                               f"everything into the earlier state. Errors faced: {e}") from e
    await post_upgrade(client, new_cfg, out)
    out(f"\n[upgrade/successful] SUCCESS! Your cluster was upgraded to {new_version!r}. Enjoy!\n\n"
        "[upgrade/kubelet] Now that your control plane is upgraded, please proceed with upgrading your kubelets "
        "in turn.")
    return new_cfg


async def post_upgrade(client, cfg, out=print):
    await P.phase_upload_config(client, cfg)
    out("[uploadconfig] Storing the configuration used in ConfigMap \"kubeadm-config\" in the \"kube-system\" Namespace")
    await P.phase_bootstrap_token_rbac(client)
    out("[bootstraptoken] Configured RBAC rules to allow Node Bootstrap tokens to post CSRs and auto-approve them")
    await P.phase_addons(client, cfg, update=True)
    out(f"[addons] Applied essential addons: kube-proxy, amd-gpu-device-plugin ({cfg['kubernetesVersion']})")


# ------------------------------------------------------------------------------------ plan
async def plan(client, cfg, out=print):
    """-> the suggested target version, or None when the cluster is up to date."""
    cluster, kubeadm_v, kubelets = await versions(client)
    out(f"[upgrade/versions] Cluster version: {cluster}")
    out(f"[upgrade/versions] kubeadm version: {kubeadm_v}")
    target = kubeadm_v if Version(cluster) < Version(kubeadm_v) else None
    if target is None:
        out("\nAwesome, you're up-to-date! Enjoy!")
        return None
    out("\nComponents that must be upgraded manually after you have upgraded the control plane with "
        "'kubeadm upgrade apply':")
    out(f"{'COMPONENT':<12}{'CURRENT':<22}AVAILABLE")
    first = True
    for v, n in sorted(kubelets.items()):
        out(f"{'Kubelet' if first else '':<12}{f'{n} x {v}':<22}{target}")
        first = False
    out(f"\nUpgrade to the latest version in the v{Version(target).major}.{Version(target).minor} series:\n")
    out(f"{'COMPONENT':<24}{'CURRENT':<18}AVAILABLE")
    for name in ("API Server", "Controller Manager", "Scheduler", "Kube Proxy"):
        out(f"{name:<24}{cluster:<18}{target}")
    out(f"\nYou can now apply the upgrade by executing the following command:\n\n\tkubeadm upgrade apply {target}\n")
    return target
