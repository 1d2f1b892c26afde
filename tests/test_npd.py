"""node-problem-detector add-on: kernel-log rules (temporary → events, permanent → conditions),
amdgpu driver rules, the AMD SMI GPU monitor (ECC / xGMI links / temperature), and coexistence
with the kubelet's own node conditions (strategic merge keyed by type).

Parity: node-problem-detector v0.4 as deployed by `cluster/addons/node-problem-detector/npd.yaml`
(kernel-monitor.json rule semantics; default conditions written at start).
"""
import json

from kubernetes_amd.addons.npd import NodeProblemDetector, default_kernel_monitor, load_monitor
from kubernetes_amd.apiserver.server import APIServer
from kubernetes_amd.client.rest import Client
from kubernetes_amd.native import amdsmi


def _conds(node):
    return {c["type"]: c for c in node["status"]["conditions"]}


def test_npd_kernel_and_gpu_monitors(run, tmp_path):
    klog = tmp_path / "kern.log"
    klog.write_text("amdgpu 0000:05:00.0: amdgpu: 3 uncorrectable hardware errors detected in UMC block\n")  # old: skipped

    async def main():
        s = APIServer()
        c = Client(f"http://127.0.0.1:{await s.start()}")
        smi = amdsmi.SMI(amdsmi.fixture_file(8, seed="npd"))
        try:
            await c.create("nodes", {"metadata": {"name": "mi355x-0"}, "status": {"conditions": [
                {"type": "Ready", "status": "True", "reason": "KubeletReady", "message": "ok"}]}})
            npd = NodeProblemDetector(c, "mi355x-0", [default_kernel_monitor(str(klog))], smi=smi)
            await npd.start()
            npd._task.cancel()
            await npd.check_once()
            cd = _conds(await c.get("nodes", "mi355x-0"))
            assert cd["Ready"]["status"] == "True"                       # kubelet's condition kept
            assert cd["KernelDeadlock"]["status"] == "False" and cd["KernelDeadlock"]["reason"] == "KernelHasNoDeadlock"
            assert cd["AMDGPUHardwareError"]["status"] == "False"      # pre-existing log line not replayed
            assert cd["XGMILinkDegraded"]["status"] == "False" and cd["GPUOverheating"]["status"] == "False"

            with open(klog, "a") as f:
                f.write("amdgpu 0000:05:00.0: amdgpu: ring gfx_0.0.0 timeout, signaled seq=12, emitted seq=14\n")
                f.write("INFO: task docker:1234 blocked for more than 120 seconds.\n")
                f.write("amdgpu 0000:75:00.0: amdgpu: partial line without newl")
            await npd.check_once()
            cd = _conds(await c.get("nodes", "mi355x-0"))
            assert cd["KernelDeadlock"]["status"] == "True" and cd["KernelDeadlock"]["reason"] == "DockerHung"
            t0 = cd["KernelDeadlock"]["lastTransitionTime"]
            reasons = [e[1] for e in npd.recorder.emitted]
            assert "AMDGPURingTimeout" in reasons and "DockerHung" in reasons

            # partial line completes → RAS uncorrectable rule → permanent condition
            with open(klog, "a") as f:
                f.write("ine: RAS poison consumption detected\n")
            await npd.check_once()
            cd = _conds(await c.get("nodes", "mi355x-0"))
            assert cd["AMDGPUHardwareError"]["status"] == "True"
            assert cd["AMDGPUHardwareError"]["reason"] == "AMDGPUUncorrectableError"
            assert cd["KernelDeadlock"]["lastTransitionTime"] == t0

            # SMI monitor: xGMI link loss on GPU 3, then recovery heals the condition
            smi.fake_set_links_up(3, 5)
            await npd.check_once()
            cd = _conds(await c.get("nodes", "mi355x-0"))
            assert cd["XGMILinkDegraded"]["status"] == "True" and "GPU 3" in cd["XGMILinkDegraded"]["message"]
            smi.fake_set_links_up(3, npd._links_base[3])
            await npd.check_once()
            cd = _conds(await c.get("nodes", "mi355x-0"))
            assert cd["XGMILinkDegraded"]["status"] == "False" and cd["XGMILinkDegraded"]["reason"] == "XGMILinksUp"

            # events were written against the Node
            await npd.recorder.flush(2.0)
            evs = (await c.list("events", "default"))["items"]
            assert any(e["reason"] == "XGMILinkDown" and e["involvedObject"]["kind"] == "Node" for e in evs)
            await npd.stop()
        finally:
            await c.close()
            await s.stop()
    run(main())


def test_npd_custom_monitor_file(tmp_path):
    cfg = {"source": "docker-monitor", "logPath": str(tmp_path / "docker.log"), "lookbackLines": 1,
           "conditions": [], "rules": [{"type": "temporary", "reason": "CorruptDockerImage",
                                         "pattern": r"Error trying v2 registry: failed to register layer: rename .*"}]}
    p = tmp_path / "docker-monitor.json"
    p.write_text(json.dumps(cfg))
    m = load_monitor(str(p))
    assert m.source == "docker-monitor" and m.rules[0].reason == "CorruptDockerImage"
    (tmp_path / "docker.log").write_text("Error trying v2 registry: failed to register layer: rename /a /b: exists\n")
    npd = NodeProblemDetector(None, "n", [m])
    npd._scan_logs()          # lookback: the existing line is read
    assert npd.recorder.emitted[0][1] == "CorruptDockerImage"


def test_parse_kmsg_record():
    from kubernetes_amd.addons.npd import parse_kmsg_record
    rec = (b"3,1234,5678901,-;amdgpu 0000:05:00.0: amdgpu: ring gfx_0.0.0 timeout, signaled seq=1\n"
           b" SUBSYSTEM=pci\n DEVICE=+pci:0000:05:00.0\n")
    assert parse_kmsg_record(rec) == ["amdgpu 0000:05:00.0: amdgpu: ring gfx_0.0.0 timeout, signaled seq=1"]
    assert parse_kmsg_record(b"6,7,8,c;tab\\x09here\n") == ["tab\there"]


def test_npd_reads_record_device(tmp_path, monkeypatch):
    """/dev/kmsg reads as size 0: the monitor must read it record by record."""
    import os

    from kubernetes_amd.addons import npd as npd_mod
    fifo = str(tmp_path / "kmsg")
    os.mkfifo(fifo)
    monkeypatch.setattr(npd_mod, "_is_char_device", lambda p: p == fifo)
    wfd = None
    det = NodeProblemDetector(None, "n", [default_kernel_monitor(fifo)])
    try:
        assert det._new_lines(det.monitors[0]) == []          # opens non-blocking, nothing yet
        wfd = os.open(fifo, os.O_WRONLY | os.O_NONBLOCK)
        os.write(wfd, b"3,99,100,-;amdgpu 0000:75:00.0: amdgpu: GPU reset(2) failed\n SUBSYSTEM=pci\n")
        det._scan_logs()
        c = det.conditions["AMDGPUHardwareError"]
        assert c["status"] == "True" and c["reason"] == "AMDGPUResetFailed"
        assert "SUBSYSTEM" not in c["message"]
    finally:
        det.close()
        if wfd is not None:
            os.close(wfd)


def test_npd_daemonset_argv_reaches_apiserver(monkeypatch):
    """The add-on manifest's own command line must parse and point at a reachable API server
    even without KUBERNETES_SERVICE_HOST (argparse used to exit)."""
    from kubernetes_amd.addons.manager import default_addons
    from kubernetes_amd.addons.npd import apiserver_url, build_detector, parse_args
    monkeypatch.delenv("KUBERNETES_SERVICE_HOST", raising=False)
    monkeypatch.delenv("KUBERNETES_MASTER", raising=False)
    ds = [o for o in default_addons() if o["metadata"]["name"] == "node-problem-detector"][0]
    cmd = ds["spec"]["template"]["spec"]["containers"][0]["command"]
    i = cmd.index("kubernetes_amd.cmd.npd")
    args = parse_args(cmd[i + 1:] + ["--smi-fixture", amdsmi.fixture_file(2, seed="npdargv")])
    client, det = build_detector(args)
    assert client.url.startswith("http://127.0.0.1:8080")
    assert det.monitors[0].log_path == "/var/log/kern.log"
    assert apiserver_url(None, {}) == "http://127.0.0.1:8080"
    assert apiserver_url(None, {"KUBERNETES_SERVICE_HOST": "10.96.0.1", "KUBERNETES_SERVICE_PORT": "443"}) == "http://127.0.0.1:8080"
    assert apiserver_url(None, {"KUBERNETES_MASTER": "http://10.0.0.1:8080"}) == "http://10.0.0.1:8080"
    dp = [o for o in default_addons() if o["metadata"]["name"] == "amd-gpu-device-plugin"][0]
    assert dp["spec"]["template"]["spec"]["volumes"][0]["hostPath"]["path"] == "/var/lib/kubelet/device-plugin"
