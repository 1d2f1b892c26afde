"""Multi-GPU checks that need a node with >= 4 MI355X (skipped on a smaller box).

* the plugin's published xGMI cliques (`amd.com/xgmi-node` + `amd.com/xgmi-peers`, from
  `amdsmi_topo_get_link_type`) agree with what HIP reports: two devices published as linked
  must be peer-accessible (`hipDeviceCanAccessPeer`, via torch), and on a fully connected
  MI355X hive every pair is;
* the [Feature:MultiGPU] e2e spec on the real node: a 4-GPU pod with
  `amd.com/xgmi-policy: required` runs the `xgmi-probe` RCCL all-reduce, every element of every
  rank verified on the GPU and the bus bandwidth above the xGMI floor.
"""
import pytest

pytestmark = pytest.mark.gpu


def _need(n):
    """Skip unless this box has n GPUs (the driver's GPU tier is a one-GPU box)."""
    import torch
    if not torch.cuda.is_available() or torch.cuda.device_count() < n:
        pytest.skip(f"needs >= {n} GPUs")


def test_published_cliques_match_hip_peer_access():
    _need(4)
    import torch
    from kubernetes_amd.deviceplugin.amdgpu import gpu_attributes, xgmi_peer_map
    from kubernetes_amd.api import core
    from kubernetes_amd.native import amdsmi
    smi = amdsmi.SMI()
    gpus = smi.gpus()
    peers = xgmi_peer_map(smi, gpus)
    attrs = {g.index: gpu_attributes(g, None, peers[g.index]) for g in gpus}
    hip = {g.index: g.hip_id if g.hip_id >= 0 else g.index for g in gpus}
    node = {(attrs[i][core.ATTR_HIVE], int(attrs[i][core.ATTR_XGMI_NODE])): i for i in attrs}
    checked = 0
    for i, a in attrs.items():
        mask = int(a[core.ATTR_XGMI_PEERS], 16)
        for (hive, k), j in node.items():
            if j == i or hive != a[core.ATTR_HIVE] or not (mask >> k) & 1:
                continue
            assert torch.cuda.can_device_access_peer(hip[i], hip[j]), (i, j, a)
            checked += 1
    print("linked pairs published and peer-accessible:", checked)
    assert checked >= 4 * 3, checked
    # one hive of fully connected MI355X packages: every pair is published as linked
    if len({a[core.ATTR_HIVE] for a in attrs.values()}) == 1 and len(attrs) == torch.cuda.device_count():
        assert checked == len(attrs) * (len(attrs) - 1)


def test_multigpu_e2e_spec_on_real_mi355x(run):
    _need(4)
    from kubernetes_amd.cluster import LocalCluster
    from kubernetes_amd.e2e import specs  # noqa: F401
    from kubernetes_amd.e2e.framework import run_specs

    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=8, runtime="process", real_gpus=True, kubelet_http=True) as cl:
            res = await run_specs(cl.url, focus="Feature:MultiGPU", timeout=240)
        assert len(res) == 1 and res[0].ok and not res[0].skipped, res[0].error if res else "no spec ran"
    run(main(), timeout=300)


HIP_PROBE = r'''
import ctypes, glob, json, os
out = {"open": {}}
for p in sorted(glob.glob("/dev/dri/renderD*")):
    try:
        os.close(os.open(p, os.O_RDWR))
        out["open"][os.path.basename(p)] = "OPEN"
    except OSError as e:
        out["open"][os.path.basename(p)] = __import__("errno").errorcode.get(e.errno, str(e.errno))
hsa = ctypes.CDLL("libhsa-runtime64.so.1")
out["hsa_init"] = hsa.hsa_init()
if out["hsa_init"] == 0:
    hsa.hsa_shut_down()
    hip = ctypes.CDLL("libamdhip64.so")
    n = ctypes.c_int(-1)
    out["hipGetDeviceCount"] = hip.hipGetDeviceCount(ctypes.byref(n))
    out["devices"] = n.value
    if n.value == 1:
        a = ctypes.POINTER(ctypes.c_float)()
        out["hipMalloc"] = hip.hipMalloc(ctypes.byref(a), ctypes.c_size_t(1 << 20))
        out["hipFree"] = hip.hipFree(a)
print("HIP " + json.dumps(out, sort_keys=True))
'''


def confinement_problems(res, mine, shim=True):
    """What is wrong with one confined container's probe output `res` (HIP_PROBE) when it was
    given the render node `mine` (None: no GPU) under kamd-runc's Landlock tier.

    With the errno shim (the default, `kamd.io/devshim` unset or "true") every sibling render
    node reads EPERM — as under a device cgroup — and ROCr starts with exactly the allowed GPU;
    with `kamd.io/devshim: "false"` siblings read raw Landlock EACCES, which ROCr's thunk treats
    as fatal, so hsa_init fails (HSA_STATUS_ERROR_OUT_OF_RESOURCES on this pool, round 5)."""
    out = []
    opened = res.get("open") or {}
    if mine is not None and opened.get(mine) != "OPEN":
        out.append(f"own node {mine} not OPEN: {opened.get(mine)}")
    want = "EPERM" if shim else "EACCES"
    bad = {n: v for n, v in opened.items() if n != mine and v != want}
    if bad:
        out.append(f"sibling render nodes should read {want}: {bad}")
    siblings = [n for n in opened if n != mine]
    if shim:
        if res.get("hsa_init") != 0:
            out.append(f"hsa_init failed under the shim: {res.get('hsa_init')}")
        elif mine is not None and (res.get("hipGetDeviceCount") != 0 or res.get("devices") != 1
                                   or res.get("hipMalloc") != 0):
            out.append(f"HIP should see exactly its one GPU and allocate: {res}")
    elif siblings and res.get("hsa_init") == 0:
        out.append("raw EACCES on siblings should fail hsa_init")
    return out


def _run_probe(tmp_path, label, devices, shim):
    import json
    import subprocess
    import sys
    from kubernetes_amd.kubelet.runtime import process as proc_rt
    probe = tmp_path / "hip_probe.py"
    probe.write_text(HIP_PROBE)
    b = tmp_path / label
    b.mkdir()
    ann = {"kamd.io/isolation-tier": "landlock", "kamd.io/landlock-dir": "/dev/dri"}
    if not shim:
        ann["kamd.io/devshim"] = "false"
    spec = {"process": {"args": [sys.executable, str(probe)], "cwd": "/",
                        "env": ["PATH=/usr/bin:/bin", "HSA_ENABLE_IPC_MODE_LEGACY=0", "LD_LIBRARY_PATH=/opt/rocm/lib"]},
            "root": {"path": "/"}, "mounts": [], "annotations": ann,
            "linux": {"devices": [{"path": d} for d in devices], "namespaces": []}}
    (b / "config.json").write_text(json.dumps(spec))
    r = subprocess.run([proc_rt.KAMD_RUNC, "run", "--bundle", str(b)], capture_output=True, text=True, timeout=120)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("HIP ")]
    assert r.returncode == 0 and line, (label, r.stdout[-1500:], r.stderr[-1500:])
    return json.loads(line[0][4:])


def test_landlock_pod_on_a_multi_gpu_node_sees_exactly_its_gpu(tmp_path):
    """Confinement on a real multi-GPU node (skips on the one-GPU lease): for every GPU k, a
    Landlock-tier container allowed only renderD(k) — with kamd-runc's default errno shim —
    reads EPERM on every sibling render node, and HIP initialises with exactly one device and
    allocates on it. This is the case the one-GPU lease cannot show: ROCr must skip the denied
    siblings rather than fail to start. The same container with the shim opted out reads raw
    EACCES on the siblings and ROCr's hsa_init fails, which is why the shim is the default."""
    import glob
    import os
    from kubernetes_amd.kubelet.runtime import process as proc_rt
    nodes = sorted(glob.glob("/dev/dri/renderD*"))
    if len(nodes) < 2:
        pytest.skip(f"needs >= 2 render nodes (this host has {len(nodes)})")
    if proc_rt.runc_features().get("tier") != "landlock":
        pytest.skip("this host is not on the Landlock tier")
    for k, node in enumerate(nodes):
        res = _run_probe(tmp_path, f"b{k}", [node], shim=True)
        print("GPU", k, node, res)
        assert confinement_problems(res, os.path.basename(node), shim=True) == [], res
    raw = _run_probe(tmp_path, "raw", [nodes[0]], shim=False)
    print("RAW", nodes[0], raw)
    assert confinement_problems(raw, os.path.basename(nodes[0]), shim=False) == [], raw
