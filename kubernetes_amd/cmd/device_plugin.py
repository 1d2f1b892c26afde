"""amd.com/gpu device plugin daemon (+ optional amd-smi Prometheus exporter).

    python -m kubernetes_amd.cmd.device_plugin --plugins-dir /var/lib/kubelet/device-plugin/plugins
"""
from __future__ import annotations

import argparse

from ..deviceplugin import api
from ..deviceplugin.amdgpu import AMDGPUPlugin
from ..native import amdsmi
from ._common import run_until_signal, setup_logging


def main(argv=None):
    ap = argparse.ArgumentParser("amdgpu-device-plugin")
    ap.add_argument("--plugins-dir", default=api.DEVICE_PLUGINS_PATH)
    ap.add_argument("--socket-name", default="amdgpu.sock")
    ap.add_argument("--fixture", default=None, help="fake AMD SMI fixture (JSON) instead of the real GPUs")
    ap.add_argument("--fake-gpus", type=int, default=0, help="generate an N x MI355X fixture")
    ap.add_argument("--health-interval", type=float, default=5.0)
    ap.add_argument("--rocm-mount", default=None, help="bind the ROCm userspace read-only into GPU containers")
    ap.add_argument("--exporter-port", type=int, default=None)
    ap.add_argument("--node-name", default="")
    ap.add_argument("--burn-in", action="store_true",
                    help="gate every GPU on the HIP acceptance test (vector_add, MFMA GEMM, HBM copy) before offering it")
    ap.add_argument("--burn-in-min-tflops", type=float, default=700.0)
    ap.add_argument("--burn-in-min-hbm-gbps", type=float, default=3000.0)
    ap.add_argument("--burn-in-min-fp8-tflops", type=float, default=1400.0,
                    help="fp8 (e4m3, block-scaled MFMA) GEMM floor; 0 skips the fp8 step")
    ap.add_argument("--xgmi-link-probe", action="store_true",
                    help="measure peer copies between the node's GPUs (xgmi-probe --p2p) after burn-in; "
                         "links below --xgmi-link-min-gbps leave the published link graph")
    ap.add_argument("--xgmi-link-min-gbps", type=float, default=25.0)
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    setup_logging(a.v)

    async def start():
        fixture = a.fixture or (amdsmi.fixture_file(a.fake_gpus) if a.fake_gpus else None)
        smi = amdsmi.SMI(fixture=fixture)
        burn_in = None
        if a.burn_in:
            from ..deviceplugin.burnin import BurnIn
            burn_in = BurnIn(min_tflops=a.burn_in_min_tflops, min_hbm_gbps=a.burn_in_min_hbm_gbps,
                             min_fp8_tflops=a.burn_in_min_fp8_tflops, fp8=a.burn_in_min_fp8_tflops > 0)
        probe = None
        if a.xgmi_link_probe and not smi.is_fake:
            from ..deviceplugin.linkprobe import run_probe
            probe = run_probe
        p = AMDGPUPlugin(a.plugins_dir, smi=smi, socket_name=a.socket_name, health_interval=a.health_interval,
                         rocm_mount=a.rocm_mount, burn_in=burn_in, link_probe=probe,
                         link_min_gbps=a.xgmi_link_min_gbps)
        await p.start()
        print(f"amd.com/gpu plugin serving {len(p.gpus)} GPU(s) on {p.socket_path}", flush=True)
        if a.exporter_port is not None:
            from ..monitoring.exporter import AMDSMIExporter
            ex = AMDSMIExporter(smi, a.node_name, health_fn=lambda i: p._health.get(i))
            port = await ex.start("0.0.0.0", a.exporter_port)
            print(f"amd-smi exporter on :{port}", flush=True)
        return p

    run_until_signal(start)


if __name__ == "__main__":
    main()
