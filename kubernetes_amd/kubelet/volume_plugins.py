"""Network and block volume plugins: nfs, cephfs, glusterfs, iscsi, fc, rbd — the in-tree
plugins of `pkg/volume/{nfs,cephfs,glusterfs,iscsi,fc,rbd}` that an on-prem MI355X cluster uses for
datasets and checkpoints (the cloud-disk plugins are out of scope).

Each plugin turns its volume source into host commands run through a `Mounter` (`pkg/util/mount`):
`mount -t <fstype> -o <options> <source> <target>` for the file systems, and for block devices the
attach step (iscsiadm discovery + login, `rbd map`, FC device lookup) then
`SafeFormatAndMount` (`blkid` probe, `mkfs.<fstype>` only on a device with no file system and
no partition table, then mount). The kubelet runs them as root on the host; a container sees the
mounted directory through its bind mount. `FakeMounter` records the commands (the reference's
`mount.FakeMounter` / `exec.FakeExec` tests).

Parity notes per plugin:
  * nfs (`nfs.go` SetUpAt): `<server>:<path>` (IPv6 servers bracketed), `ro` for readOnly, the
    PV's mountOptions;
  * cephfs (`cephfs.go`): `<mon1,mon2,...>:<path or />`, `name=<user or admin>`, the key from
    `secretRef` (`key` entry) as `secret=` or `secretfile=<secretFile or /etc/ceph/<user>.secret>`;
  * glusterfs (`glusterfs.go`): the hosts of the `endpoints` object, `<host>:<path>`,
    `backup-volfile-servers=<others>`, `log-file=` under the plugin dir;
  * iscsi (`iscsi_util.go` AttachDisk): for the portal and each extra `portals` entry
    `iscsiadm -m discoverydb -t sendtargets -p <portal> -I <iface> -o new|--discover`, then
    `iscsiadm -m node -p <portal> -T <iqn> -I <iface> --login` (CHAP settings first when
    `chapAuthSession`), device `/dev/disk/by-path/ip-<portal>-iscsi-<iqn>-lun-<lun>`; logout on
    detach;
  * fc (`fc_util.go`): `/dev/disk/by-path/*-fc-0x<wwn>-lun-<lun>` for the targetWWNs, or
    `/dev/disk/by-id/scsi-<wwid>`;
  * rbd (`rbd_util.go`): `rbd map <pool>/<image> --id <user> -m <mons> --key=<secret>` (or
    `-k <keyring>`), the device it prints; `rbd unmap` on detach.
"""
from __future__ import annotations

import asyncio
import base64
import glob
import ipaddress
import os

NETWORK_KINDS = ("nfs", "cephfs", "glusterfs", "iscsi", "fc", "rbd")


class MountError(Exception):
    pass


class Mounter:
    """Runs host mount-related commands (the kubelet is root on a real node)."""

    async def run(self, argv, timeout=120.0) -> tuple[int, str]:
        try:
            p = await asyncio.create_subprocess_exec(*argv, stdout=asyncio.subprocess.PIPE,
                                                     stderr=asyncio.subprocess.STDOUT)
        except OSError as e:
            return 127, str(e)
        try:
            out, _ = await asyncio.wait_for(p.communicate(), timeout)
        except asyncio.TimeoutError:
            p.kill()
            await p.wait()
            return 124, "timeout"
        return p.returncode, out.decode(errors="replace")

    async def mount(self, source, target, fstype, options=()):
        os.makedirs(target, exist_ok=True)
        argv = ["mount"] + (["-t", fstype] if fstype else []) + (["-o", ",".join(options)] if options else []) + \
            [source, target]
        rc, out = await self.run(argv)
        if rc != 0:
            raise MountError(f"mount failed: {' '.join(argv)}: {out.strip()}")

    async def unmount(self, target):
        rc, out = await self.run(["umount", target])
        if rc != 0 and self.is_mount_point(target):
            raise MountError(f"umount {target}: {out.strip()}")

    def is_mount_point(self, path) -> bool:
        return os.path.ismount(path)

    def exists(self, path) -> bool:
        return os.path.exists(path)

    def glob(self, pattern):
        return sorted(glob.glob(pattern))


class FakeMounter(Mounter):
    """Records commands; `results` maps an argv prefix (tuple) to (rc, output); `devices` is the
    set of device paths that "exist" (after an attach command, see `appear`)."""

    def __init__(self):
        self.log: list = []
        self.mounts: dict[str, tuple] = {}
        self.results: dict[tuple, tuple] = {}
        self.devices: set = set()
        self.appear: dict[tuple, str] = {}     # argv prefix -> device path created by that command

    async def run(self, argv, timeout=120.0):
        self.log.append(list(argv))
        for k, dev in self.appear.items():
            if tuple(argv[:len(k)]) == k:
                self.devices.add(dev)
        for k in sorted(self.results, key=len, reverse=True):
            if tuple(argv[:len(k)]) == k:
                return self.results[k]
        if argv[0] == "mount":
            self.mounts[argv[-1]] = (argv[-2], argv)
        elif argv[0] == "umount":
            self.mounts.pop(argv[-1], None)
        return 0, ""

    def is_mount_point(self, path):
        return path in self.mounts

    def exists(self, path):
        return path in self.devices

    def glob(self, pattern):
        import fnmatch
        return sorted(d for d in self.devices if fnmatch.fnmatch(d, pattern))


def _host(server: str) -> str:
    try:
        if ipaddress.ip_address(server).version == 6:
            return f"[{server}]"
    except ValueError:
        pass
    return server


class PluginContext:
    """What a plugin needs from the kubelet: the API (secrets, endpoints), the pod namespace,
    the mounter, and a directory for plugin state (log files, keyrings)."""

    def __init__(self, client, namespace, mounter: Mounter, plugin_dir, mount_options=()):
        self.client, self.namespace, self.mounter = client, namespace, mounter
        self.plugin_dir = plugin_dir
        self.mount_options = list(mount_options)

    async def secret_value(self, ref, key):
        ns = ref.get("namespace") or self.namespace
        s = await self.client.get("secrets", ref["name"], ns)
        v = (s.get("data") or {}).get(key)
        if v is None:
            raise MountError(f"secret {ns}/{ref['name']} has no key {key!r}")
        return base64.b64decode(v).decode()


# -- file systems --------------------------------------------------------------------------------
async def mount_nfs(src, target, ctx):
    opts = list(ctx.mount_options) + (["ro"] if src.get("readOnly") else [])
    await ctx.mounter.mount(f"{_host(src['server'])}:{src['path']}", target, "nfs", opts)
    return {"target": target}


async def mount_cephfs(src, target, ctx):
    user = src.get("user") or "admin"
    opts = [f"name={user}"]
    if src.get("secretRef"):
        opts.append("secret=" + await ctx.secret_value(src["secretRef"], "key"))
    else:
        opts.append("secretfile=" + (src.get("secretFile") or f"/etc/ceph/{user}.secret"))
    if src.get("readOnly"):
        opts.append("ro")
    mons = ",".join(src.get("monitors") or ())
    await ctx.mounter.mount(f"{mons}:{src.get('path') or '/'}", target, "ceph", ctx.mount_options + opts)
    return {"target": target}


async def mount_glusterfs(src, target, ctx):
    ep = await ctx.client.get("endpoints", src["endpoints"], ctx.namespace)
    hosts = [a["ip"] for s in ep.get("subsets") or () for a in s.get("addresses") or ()]
    if not hosts:
        raise MountError(f"glusterfs: endpoints {ctx.namespace}/{src['endpoints']} has no addresses")
    os.makedirs(ctx.plugin_dir, exist_ok=True)
    log = os.path.join(ctx.plugin_dir, os.path.basename(target.rstrip("/")) + "-glusterfs.log")
    err = None
    for i, h in enumerate(hosts):
        others = hosts[:i] + hosts[i + 1:]
        opts = list(ctx.mount_options) + [f"log-file={log}"] + \
            ([f"backup-volfile-servers={':'.join(others)}"] if others else []) + (["ro"] if src.get("readOnly") else [])
        try:
            await ctx.mounter.mount(f"{h}:{src['path']}", target, "glusterfs", opts)
            return {"target": target}
        except MountError as e:
            err = e
    raise MountError(f"glusterfs: no server of {src['endpoints']} mounted {src['path']}: {err}")


# -- block devices ---------------------------------------------------------------------------------
async def _wait_device(ctx, candidates_fn, timeout=10.0):
    end = asyncio.get_running_loop().time() + timeout
    while True:
        devs = candidates_fn()
        if devs:
            return devs[0]
        if asyncio.get_running_loop().time() > end:
            return None
        await asyncio.sleep(0.2)


async def format_and_mount(ctx, device, target, fstype, read_only, options=()):
    """`SafeFormatAndMount`: format only a device with neither a file system nor a partition
    table, never a read-only one."""
    fstype = fstype or "ext4"
    rc, out = await ctx.mounter.run(["blkid", "-p", "-s", "TYPE", "-s", "PTTYPE", "-o", "export", device])
    if rc == 2 and not read_only:      # blkid: nothing found
        argv = [f"mkfs.{fstype}"] + (["-F", "-m0"] if fstype.startswith("ext") else []) + [device]
        rc2, out2 = await ctx.mounter.run(argv)
        if rc2 != 0:
            raise MountError(f"format {device} as {fstype}: {out2.strip()}")
    elif rc != 0 and rc != 2:
        raise MountError(f"blkid {device}: {out.strip()}")
    elif "PTTYPE=" in out and "TYPE=" not in out.replace("PTTYPE=", ""):
        raise MountError(f"{device} has a partition table and no file system: refusing to format it")
    await ctx.mounter.mount(device, target, fstype, list(options) + (["ro"] if read_only else []))


def _iscsi_device(portal, iqn, lun):
    p = portal if ":" in portal.rsplit("]", 1)[-1] else portal + ":3260"
    return f"/dev/disk/by-path/ip-{p}-iscsi-{iqn}-lun-{lun}"


async def mount_iscsi(src, target, ctx):
    iface = src.get("iscsiInterface") or "default"
    iqn, lun = src["iqn"], int(src.get("lun", 0))
    portals = [src["targetPortal"]] + list(src.get("portals") or ())
    chap = {}
    if src.get("chapAuthDiscovery") or src.get("chapAuthSession"):
        if not src.get("secretRef"):
            raise MountError("iscsi: CHAP authentication needs a secretRef")
        for k in ("node.session.auth.username", "node.session.auth.password",
                  "discovery.sendtargets.auth.username", "discovery.sendtargets.auth.password"):
            try:
                chap[k] = await ctx.secret_value(src["secretRef"], k)
            except MountError:
                pass
    device = None
    for portal in portals:
        p = portal if ":" in portal.rsplit("]", 1)[-1] else portal + ":3260"
        base = ["iscsiadm", "-m", "discoverydb", "-t", "sendtargets", "-p", p, "-I", iface]
        await ctx.mounter.run(base + ["-o", "new"])
        if src.get("chapAuthDiscovery"):
            for k in ("discovery.sendtargets.auth.username", "discovery.sendtargets.auth.password"):
                if k in chap:
                    await ctx.mounter.run(base + ["-o", "update", "-n", k, "-v", chap[k]])
        rc, out = await ctx.mounter.run(base + ["--discover"])
        if rc != 0:
            continue
        node = ["iscsiadm", "-m", "node", "-p", p, "-T", iqn, "-I", iface]
        if src.get("chapAuthSession"):
            await ctx.mounter.run(node + ["-o", "update", "-n", "node.session.auth.authmethod", "-v", "CHAP"])
            for k in ("node.session.auth.username", "node.session.auth.password"):
                if k in chap:
                    await ctx.mounter.run(node + ["-o", "update", "-n", k, "-v", chap[k]])
        rc, out = await ctx.mounter.run(node + ["--login"])
        if rc != 0:
            continue
        dev = _iscsi_device(portal, iqn, lun)
        if await _wait_device(ctx, lambda: [dev] if ctx.mounter.exists(dev) else []):
            device = device or dev
    if device is None:
        raise MountError(f"iscsi: could not attach {iqn} lun {lun} through {portals}")
    await format_and_mount(ctx, device, target, src.get("fsType"), bool(src.get("readOnly")), ctx.mount_options)
    return {"target": target, "iscsi": (portals, iqn, iface)}


async def mount_fc(src, target, ctx):
    if src.get("targetWWNs"):
        lun = int(src.get("lun", 0))
        pats = [f"/dev/disk/by-path/*-fc-0x{w.lower()}-lun-{lun}" for w in src["targetWWNs"]]
    elif src.get("wwids"):
        pats = [f"/dev/disk/by-id/scsi-{w}" for w in src["wwids"]]
    else:
        raise MountError("fc: targetWWNs+lun or wwids is required")
    dev = await _wait_device(ctx, lambda: [d for p in pats for d in ctx.mounter.glob(p)])
    if dev is None:
        raise MountError(f"fc: no device for {pats}")
    await format_and_mount(ctx, dev, target, src.get("fsType"), bool(src.get("readOnly")), ctx.mount_options)
    return {"target": target}


async def mount_rbd(src, target, ctx):
    pool, image = src.get("pool") or "rbd", src["image"]
    user = src.get("user") or "admin"
    argv = ["rbd", "map", f"{pool}/{image}", "--id", user, "-m", ",".join(src.get("monitors") or ())]
    if src.get("secretRef"):
        argv.append("--key=" + await ctx.secret_value(src["secretRef"], "key"))
    else:
        argv += ["-k", src.get("keyring") or "/etc/ceph/keyring"]
    rc, out = await ctx.mounter.run(argv)
    if rc != 0:
        raise MountError(f"rbd map {pool}/{image}: {out.strip()}")
    dev = (out.strip().splitlines() or [""])[-1].strip() or f"/dev/rbd/{pool}/{image}"
    await format_and_mount(ctx, dev, target, src.get("fsType"), bool(src.get("readOnly")), ctx.mount_options)
    return {"target": target, "rbd": dev}


MOUNT = {"nfs": mount_nfs, "cephfs": mount_cephfs, "glusterfs": mount_glusterfs, "iscsi": mount_iscsi,
         "fc": mount_fc, "rbd": mount_rbd}


async def detach(ctx, state: dict, still_used=lambda key: False):
    """Unmount, then release what the attach created (iSCSI session, mapped rbd device) unless
    another mounted volume still uses it."""
    target = state["target"]
    if ctx.mounter.is_mount_point(target):
        await ctx.mounter.unmount(target)
    if "iscsi" in state and not still_used(("iscsi", state["iscsi"][1])):
        portals, iqn, iface = state["iscsi"]
        for portal in portals:
            p = portal if ":" in portal.rsplit("]", 1)[-1] else portal + ":3260"
            await ctx.mounter.run(["iscsiadm", "-m", "node", "-p", p, "-T", iqn, "-I", iface, "--logout"])
    if "rbd" in state and not still_used(("rbd", state["rbd"])):
        await ctx.mounter.run(["rbd", "unmap", state["rbd"]])
