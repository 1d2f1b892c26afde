"""Native C++ components on CPU: amdsmi shim (fake backend), OCI device helper, pause/orphan."""
import os
import signal
import subprocess
import time

import pytest

from kubernetes_amd.native import BIN_DIR
from kubernetes_amd.native import amdsmi
from kubernetes_amd.native.oci import oci_devices


def test_fake_backend_8x_mi355x():
    smi = amdsmi.SMI(fixture=amdsmi.fixture_file(8))
    assert smi.is_fake and smi.count() == 8
    g = smi.gpu(3)
    assert g.arch == "gfx950" and g.vram_total_mb == 294912 and g.compute_units == 256
    assert g.render_minor == 131 and g.market_name == "AMD Instinct MI355X"
    assert g.device_id_str.startswith("GPU-") and len(g.device_id_str) <= 63
    # all-to-all xGMI inside one hive
    topo = smi.topology()
    for i in range(8):
        for j in range(8):
            if i != j:
                assert topo[i][j].type == amdsmi.LINK_XGMI and topo[i][j].hops == 1 and topo[i][j].p2p
    m = smi.metrics(0)
    assert m.xgmi_links_up == 7 and m.ecc_uncorrectable == 0
    smi.fake_set_ecc(0, 5)
    assert smi.metrics(0).ecc_uncorrectable == 5


def test_fake_backend_two_hives():
    smi = amdsmi.SMI(fixture=amdsmi.fixture_file(8, hives=2))
    topo = smi.topology()
    assert topo[0][3].type == amdsmi.LINK_XGMI
    assert topo[0][4].type == amdsmi.LINK_PCIE and not topo[0][4].p2p


def test_fake_backend_cpx_partitions():
    """CPX mode: each MI355X package exposes 8 logical devices (one XCD, 32 CUs, 1/8 of the
    HBM, own render node) sharing the package's socket; NPS is reported per device."""
    smi = amdsmi.SMI(fixture=amdsmi.fixture_file(2, partition="CPX", memory_partition="NPS2"))
    gs = smi.gpus()
    assert len(gs) == 16 and len({g.device_id_str for g in gs}) == 16
    assert {g.render_minor for g in gs} == set(range(128, 144))
    assert [g.socket for g in gs] == [0] * 8 + [1] * 8 and [g.partition_id for g in gs[:8]] == list(range(8))
    assert all(g.compute_units == 32 and g.vram_total_mb == 294912 // 8 and g.memory_partition == "NPS2" for g in gs)
    on_pkg, off_pkg = smi.link(0, 7), smi.link(0, 8)
    assert on_pkg.hops == 0 and on_pkg.weight < off_pkg.weight and off_pkg.type == amdsmi.LINK_XGMI


def test_bad_fixture(tmp_path):
    p = tmp_path / "bad.json"
    p.write_text("{nope")
    with pytest.raises(amdsmi.SMIError):
        amdsmi.SMI(fixture=str(p))


def test_oci_devices():
    out = oci_devices(["/dev/null", "/dev/zero"], "rw")
    assert [d["path"] for d in out["devices"]] == ["/dev/null", "/dev/zero"]
    assert out["devices"][0]["type"] == "c" and out["devices"][0]["major"] == 1 and out["devices"][0]["minor"] == 3
    assert out["allow"][1] == {"allow": True, "type": "c", "major": 1, "minor": 5, "access": "rw"}
    with pytest.raises(FileNotFoundError):
        oci_devices(["/dev/null", "/etc/hostname"])


def test_pause_exits_on_sigterm():
    pause = os.path.join(BIN_DIR, "pause")
    p = subprocess.Popen([pause], stderr=subprocess.PIPE)
    time.sleep(0.2)
    assert p.poll() is None
    p.send_signal(signal.SIGTERM)
    assert p.wait(5) == 0


def test_orphan_helper_runs():
    out = subprocess.run([os.path.join(BIN_DIR, "orphan"), "0"], capture_output=True, text=True, timeout=10)
    assert out.returncode == 0 and "orphaned" in out.stdout
