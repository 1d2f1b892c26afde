"""node-problem-detector: node conditions and events from kernel logs and AMD SMI.

Parity: the `cluster/addons/node-problem-detector/npd.yaml` add-on (a DaemonSet running
node-problem-detector v0.4 with `--system-log-monitors=kernel-monitor.json,docker-monitor.json`).
Its model is kept:
  * a *system log monitor* tails a log, matches each line against rules, and reports either
    a **temporary** problem (a Warning event on the Node) or a **permanent** problem (a Node
    condition set True with the rule's reason, e.g. `KernelDeadlock`);
  * at start every monitored condition is written with its default (False) status, so a
    healed node is visibly healed after a restart;
  * conditions are re-sent every `heartbeat` seconds (lastHeartbeatTime), and
    lastTransitionTime only moves when the status flips.

MI355X additions (the part the reference's NVIDIA fork never had): rules for the `amdgpu`
kernel driver (ring timeouts, GPU resets, RAS uncorrectable/poison errors, xGMI link errors)
and an **AMD SMI monitor** that polls each GPU's uncorrectable ECC count, xGMI links up and
hotspot temperature and drives `AMDGPUHardwareError`, `XGMILinkDegraded` and `GPUOverheating`
conditions. The device plugin marks the affected GPU Unhealthy; NPD makes the node-level
problem visible to operators and to remedy controllers (`kubectl describe node`).
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import re
import stat
from dataclasses import dataclass, field

from ..api.meta import now_rfc3339
from ..client.events import EventRecorder

log = logging.getLogger("node-problem-detector")

TEMPORARY, PERMANENT = "temporary", "permanent"


@dataclass
class Rule:
    type: str                   # temporary | permanent
    reason: str
    pattern: str
    condition: str = ""         # for permanent rules
    _re: re.Pattern = field(default=None, repr=False)

    def __post_init__(self):
        self._re = re.compile(self.pattern)


@dataclass
class MonitorConfig:
    source: str                 # e.g. kernel-monitor
    log_path: str
    conditions: list            # [{"type", "reason", "message"}] defaults (status False)
    rules: list                 # [Rule]
    lookback_lines: int = 0     # lines already in the log at start are skipped unless > 0

    @classmethod
    def from_dict(cls, d, log_path=None):
        return cls(source=d.get("source", "kernel-monitor"), log_path=log_path or d.get("logPath", "/dev/kmsg"),
                   conditions=list(d.get("conditions") or []),
                   rules=[Rule(r["type"], r["reason"], r["pattern"], r.get("condition", "")) for r in d.get("rules") or []],
                   lookback_lines=int(d.get("lookbackLines", 0)))


def default_kernel_monitor(log_path="/dev/kmsg") -> MonitorConfig:
    """kernel-monitor.json of NPD v0.4 plus amdgpu driver rules."""
    return MonitorConfig.from_dict({
        "source": "kernel-monitor",
        "conditions": [
            {"type": "KernelDeadlock", "reason": "KernelHasNoDeadlock", "message": "kernel has no deadlock"},
            {"type": "AMDGPUHardwareError", "reason": "AMDGPUHasNoHardwareError", "message": "no uncorrectable GPU errors"},
        ],
        "rules": [
            {"type": TEMPORARY, "reason": "OOMKilling", "pattern": r"Kill process \d+ (.+) score \d+ or sacrifice child\nKilled process \d+ (.+) total-vm:\d+kB, anon-rss:\d+kB, file-rss:\d+kB.*|Out of memory: Kill(ed)? process \d+ .*"},
            {"type": TEMPORARY, "reason": "TaskHung", "pattern": r"task \S+:\w+ blocked for more than \w+ seconds\."},
            {"type": TEMPORARY, "reason": "UnregisterNetDevice", "pattern": r"unregister_netdevice: waiting for \w+ to become free. Usage count = \d+"},
            {"type": TEMPORARY, "reason": "KernelOops", "pattern": r"BUG: unable to handle kernel NULL pointer dereference at .*"},
            {"type": TEMPORARY, "reason": "KernelOops", "pattern": r"divide error: 0000 \[#\d+\] SMP"},
            {"type": PERMANENT, "condition": "KernelDeadlock", "reason": "AUFSUmountHung", "pattern": r"task umount\.aufs:\w+ blocked for more than \w+ seconds\."},
            {"type": PERMANENT, "condition": "KernelDeadlock", "reason": "DockerHung", "pattern": r"task docker:\w+ blocked for more than \w+ seconds\."},
            # amdgpu driver (gfx950)
            {"type": TEMPORARY, "reason": "AMDGPURingTimeout", "pattern": r"amdgpu \S+: .*ring (\S+) timeout"},
            {"type": TEMPORARY, "reason": "AMDGPUReset", "pattern": r"amdgpu \S+: .*GPU reset(\(\d+\))? (begin|succeeded)"},
            {"type": TEMPORARY, "reason": "AMDGPUPageFault", "pattern": r"amdgpu \S+: .*\[gfxhub\] page fault"},
            {"type": PERMANENT, "condition": "AMDGPUHardwareError", "reason": "AMDGPUUncorrectableError",
             "pattern": r"amdgpu \S+: .*(uncorrectable hardware error|RAS poison consumption|\d+ uncorrectable hardware errors detected)"},
            {"type": PERMANENT, "condition": "AMDGPUHardwareError", "reason": "AMDGPUResetFailed",
             "pattern": r"amdgpu \S+: .*(GPU reset\(\d+\) failed|ASIC reset failed)"},
            {"type": TEMPORARY, "reason": "XGMILinkError", "pattern": r"amdgpu \S+: .*(xgmi|XGMI).*(error|link down)"},
        ],
    }, log_path)


def _is_char_device(path) -> bool:
    try:
        return stat.S_ISCHR(os.stat(path).st_mode)
    except OSError:
        return False


def parse_kmsg_record(rec: bytes) -> list:
    """One /dev/kmsg record -> its message line(s). The header `prio,seq,ts,flags[,..];` is
    dropped; continuation lines (leading space, `KEY=value` device metadata) are skipped;
    `\\xNN` escapes the kernel applies to non-printable bytes are undone."""
    text = rec.decode(errors="replace")
    head, sep, body = text.partition(";")
    if not sep or not head[:1].isdigit():
        body = text                          # not a record header: treat as a plain line
    lines = []
    for i, ln in enumerate(body.split("\n")):
        if i > 0 and (not ln or ln.startswith(" ")):
            continue
        if "\\x" in ln:
            ln = re.sub(r"\\x([0-9a-fA-F]{2})", lambda mt: chr(int(mt.group(1), 16)), ln)
        if ln:
            lines.append(ln)
    return lines


def apiserver_url(master=None, env=None) -> str:
    """Where an add-on pod finds the API server: --master, then $KUBERNETES_MASTER, then the
    in-cluster service env ($KUBERNETES_SERVICE_HOST/_PORT; 443 is the service port that
    forwards to the secure port, so only an explicit non-443 port is used as plain HTTP),
    then the local insecure port — add-ons run hostNetwork on the control-plane node, as the
    DNS add-on assumes (`cmd/dns.py`)."""
    env = os.environ if env is None else env
    if master:
        return master
    if env.get("KUBERNETES_MASTER"):
        return env["KUBERNETES_MASTER"]
    host, port = env.get("KUBERNETES_SERVICE_HOST"), env.get("KUBERNETES_SERVICE_PORT", "443")
    if host and port not in ("443", "6443"):
        return f"http://{host}:{port}"
    return "http://127.0.0.1:8080"


class NodeProblemDetector:
    """One per node. `check_once()` (tests) or `start()` (poll loop)."""

    def __init__(self, client, node_name, monitors=(), smi=None, period=1.0, heartbeat=300.0,
                 ecc_threshold=0, max_temp_c=105):
        self.client = client
        self.node = node_name
        self.monitors = list(monitors)
        self.smi = smi
        self.period = period
        self.heartbeat = heartbeat
        self.ecc_threshold = ecc_threshold
        self.max_temp_c = max_temp_c
        self.recorder = EventRecorder(client, "node-problem-detector", host=node_name)
        self.conditions: dict[str, dict] = {}      # type -> condition
        self._dirty = True
        self._last_sent = 0.0
        self._offsets: dict[str, int] = {}
        self._kmsg: dict[str, int] = {}          # record-device path -> non-blocking fd
        self._ecc_base: dict[int, int] = {}
        self._links_base: dict[int, int] = {}
        self._task = None
        for m in self.monitors:
            for c in m.conditions:
                self._set(c["type"], "False", c["reason"], c["message"])
        if smi is not None:
            for t, r, msg in (("AMDGPUHardwareError", "AMDGPUHasNoHardwareError", "no uncorrectable GPU errors"),
                              ("XGMILinkDegraded", "XGMILinksUp", "all xGMI links are up"),
                              ("GPUOverheating", "GPUTemperatureNormal", "GPU temperatures are normal")):
                if t not in self.conditions:
                    self._set(t, "False", r, msg)
            for g in smi.gpus():
                m = smi.metrics(g.index)
                self._ecc_base[g.index] = m.ecc_uncorrectable
                self._links_base[g.index] = m.xgmi_links_up

    # -- state -----------------------------------------------------------------
    def _set(self, ctype, status, reason, message):
        now = now_rfc3339()
        old = self.conditions.get(ctype)
        if old and old["status"] == status and old["reason"] == reason and old["message"] == message:
            return False
        self.conditions[ctype] = {"type": ctype, "status": status, "reason": reason, "message": message,
                                  "lastHeartbeatTime": now,
                                  "lastTransitionTime": now if (not old or old["status"] != status) else old["lastTransitionTime"]}
        self._dirty = True
        return True

    def _node_ref(self):
        return {"kind": "Node", "apiVersion": "v1", "metadata": {"name": self.node, "uid": self.node, "namespace": ""}}

    # -- log monitors ----------------------------------------------------------
    def _new_lines(self, m: MonitorConfig):
        if m.log_path in self._kmsg or _is_char_device(m.log_path):
            return self._kmsg_lines(m)
        try:
            size = os.path.getsize(m.log_path)
        except OSError:
            return []
        off = self._offsets.get(m.log_path)
        if off is None:
            off = size
            if m.lookback_lines:
                off = 0
        if size < off:      # rotated / truncated
            off = 0
        if size == off:
            self._offsets[m.log_path] = off
            return []
        with open(m.log_path, "rb") as f:
            f.seek(off)
            data = f.read(size - off)
        # only complete lines
        cut = data.rfind(b"\n") + 1
        self._offsets[m.log_path] = off + cut
        return data[:cut].decode(errors="replace").splitlines()

    def _kmsg_lines(self, m: MonitorConfig):
        """/dev/kmsg is a record device: its size reads as 0 and every read() returns one
        record `prio,seq,ts_us,flags[,...];message\\n` followed by ` KEY=value` continuation
        lines. Open it non-blocking once, skip the backlog (unless lookback is asked: the
        kernel then replays its ring buffer from the first record), read until EAGAIN.
        NPD v0.4's kmsg watcher (`pkg/systemlogmonitor/logwatchers/kmsg`) reads it the same way."""
        fd = self._kmsg.get(m.log_path)
        if fd is None:
            try:
                fd = os.open(m.log_path, os.O_RDONLY | os.O_NONBLOCK)
            except OSError as e:
                log.warning("cannot open %s: %s", m.log_path, e)
                return []
            if not m.lookback_lines:
                try:
                    os.lseek(fd, 0, os.SEEK_END)        # SEEK_END = "after the newest record"
                except OSError:
                    pass
            self._kmsg[m.log_path] = fd
        out = []
        while True:
            try:
                rec = os.read(fd, 8192)
            except BlockingIOError:
                break
            except OSError as e:
                if e.errno == 32:      # EPIPE: records were overwritten before we read them; continue
                    continue
                log.warning("reading %s failed: %s", m.log_path, e)
                break
            if not rec:
                break
            out.extend(parse_kmsg_record(rec))
        return out

    def close(self):
        for fd in self._kmsg.values():
            try:
                os.close(fd)
            except OSError:
                pass
        self._kmsg.clear()

    def _scan_logs(self):
        for m in self.monitors:
            for line in self._new_lines(m):
                for r in m.rules:       # every rule sees every line (TaskHung + DockerHung)
                    if not r._re.search(line):
                        continue
                    if r.type == TEMPORARY:
                        self.recorder.event(self._node_ref(), "Warning", r.reason, line.strip())
                    else:
                        if self._set(r.condition, "True", r.reason, line.strip()):
                            self.recorder.event(self._node_ref(), "Warning", r.reason, line.strip())

    # -- AMD SMI monitor -------------------------------------------------------
    def _scan_smi(self):
        bad_ecc, down, hot = [], [], []
        for g in self.smi.gpus():
            m = self.smi.metrics(g.index)
            if m.ecc_uncorrectable - self._ecc_base.get(g.index, 0) > self.ecc_threshold:
                bad_ecc.append(f"GPU {g.index} ({g.bdf}): {m.ecc_uncorrectable} uncorrectable ECC errors")
            if m.xgmi_links_up < self._links_base.get(g.index, 0):
                down.append(f"GPU {g.index} ({g.bdf}): {m.xgmi_links_up}/{m.xgmi_links_total} xGMI links up")
            if self.max_temp_c and m.temp_hotspot_c >= self.max_temp_c:
                hot.append(f"GPU {g.index} ({g.bdf}): hotspot {m.temp_hotspot_c} C")
        for ctype, items, reason_bad, reason_ok, ok_msg in (
                ("AMDGPUHardwareError", bad_ecc, "AMDGPUUncorrectableECC", "AMDGPUHasNoHardwareError", "no uncorrectable GPU errors"),
                ("XGMILinkDegraded", down, "XGMILinkDown", "XGMILinksUp", "all xGMI links are up"),
                ("GPUOverheating", hot, "GPUHotspotOverLimit", "GPUTemperatureNormal", "GPU temperatures are normal")):
            cur = self.conditions.get(ctype, {})
            if items:
                if self._set(ctype, "True", reason_bad, "; ".join(items)):
                    self.recorder.event(self._node_ref(), "Warning", reason_bad, "; ".join(items))
            elif cur.get("status") == "True" and cur.get("reason") == reason_bad:
                # SMI-driven problems heal when the counters do; log-driven ones stay until restart
                self._set(ctype, "False", reason_ok, ok_msg)

    # -- exporter --------------------------------------------------------------
    async def _sync(self, now):
        if not self._dirty and now - self._last_sent < self.heartbeat:
            return
        hb = now_rfc3339()
        for c in self.conditions.values():
            c["lastHeartbeatTime"] = hb
        conds = [dict(c) for c in self.conditions.values()]
        # strategic merge keyed by condition type: the kubelet's own conditions are left alone
        await self.client.patch("nodes", self.node, {"status": {"conditions": conds}}, patch_type="strategic",
                                subresource="status")
        self._dirty = False
        self._last_sent = now

    async def check_once(self):
        self._scan_logs()
        if self.smi is not None:
            self._scan_smi()
        await self._sync(asyncio.get_running_loop().time())

    async def _loop(self):
        while True:
            try:
                await self.check_once()
            except Exception as e:  # noqa: BLE001 - keep monitoring
                log.warning("problem detection pass failed: %s", e)
            await asyncio.sleep(self.period)

    async def start(self):
        self.recorder.start()
        for m in self.monitors:       # skip what is already in the logs unless lookback is asked
            if not m.lookback_lines:
                self._new_lines(m)
        self._task = asyncio.ensure_future(self._loop())
        return self

    async def stop(self):
        if self._task:
            self._task.cancel()
            try:
                await self._task
            except asyncio.CancelledError:
                pass
        await self.recorder.flush(1.0)
        self.recorder.stop()
        self.close()


def load_monitor(path, log_path=None) -> MonitorConfig:
    with open(path) as f:
        return MonitorConfig.from_dict(json.load(f), log_path)


def parse_args(argv=None):
    import argparse
    ap = argparse.ArgumentParser("node-problem-detector")
    ap.add_argument("--apiserver-override", "--master", dest="master", default=None,
                    help="API server URL (default: $KUBERNETES_MASTER, the in-cluster service, or http://127.0.0.1:8080)")
    ap.add_argument("--kubeconfig", default=None)
    ap.add_argument("--hostname-override", default=os.environ.get("NODE_NAME") or os.uname().nodename)
    ap.add_argument("--system-log-monitors", default="", help="comma-separated monitor JSON files")
    ap.add_argument("--kernel-log", default="/dev/kmsg",
                    help="log for the built-in kernel monitor: /dev/kmsg (record device) or a text log such as /var/log/kern.log")
    ap.add_argument("--amd-smi", action="store_true", help="enable the AMD SMI GPU monitor")
    ap.add_argument("--smi-fixture", default=None)
    ap.add_argument("--period", type=float, default=1.0)
    return ap.parse_args(argv)


def build_detector(args):
    """argv -> (client, NodeProblemDetector) without starting anything (tests use this with the
    DaemonSet manifest's own command line)."""
    from ..client.clientcmd import client_from
    from ..client.rest import Client
    from ..native import amdsmi
    mons = [load_monitor(p) for p in args.system_log_monitors.split(",") if p] or [default_kernel_monitor(args.kernel_log)]
    for m in mons:
        if not os.path.exists(m.log_path):
            log.warning("log %s does not exist yet; the monitor starts reading once it appears", m.log_path)
    smi = amdsmi.SMI(args.smi_fixture) if (args.amd_smi or args.smi_fixture) else None
    client = client_from(args.kubeconfig) if args.kubeconfig else Client(apiserver_url(args.master))
    return client, NodeProblemDetector(client, args.hostname_override, mons, smi, args.period)


def main(argv=None):
    import sys
    args = parse_args(argv)
    logging.basicConfig(level=logging.INFO, stream=sys.stderr)

    async def run():
        _, det = build_detector(args)
        npd = await det.start()
        try:
            await asyncio.Event().wait()
        finally:
            await npd.stop()
    asyncio.run(run())


if __name__ == "__main__":
    main()
