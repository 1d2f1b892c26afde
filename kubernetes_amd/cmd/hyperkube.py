"""hyperkube: every component behind one entry point (`cmd/hyperkube`, `pkg/hyperkube`).

    python -m kubernetes_amd.cmd.hyperkube <component> [flags...]

The component is taken from the first argument, or from the program name when invoked through
a symlink named after it (`kube-apiserver`, `kubelet`, ...), as the reference does.
"""
import importlib
import os
import sys

COMPONENTS = {
    "apiserver": "apiserver", "kube-apiserver": "apiserver",
    "controller-manager": "controller_manager", "kube-controller-manager": "controller_manager",
    "scheduler": "scheduler", "kube-scheduler": "scheduler",
    "kubelet": "kubelet",
    "proxy": "proxy", "kube-proxy": "proxy",
    "kubectl": "kubectl",
    "kubeadm": "kubeadm",
    "dns": "dns", "kube-dns": "dns",
    "addon-manager": "addon_manager", "kube-addon-manager": "addon_manager",
    "cri": "cri", "kamd-cri": "cri",
    "device-plugin": "device_plugin", "amd-gpu-device-plugin": "device_plugin",
    "amd-smi-exporter": "amd_smi_exporter",
    "dashboard": "dashboard",
    "hollow-node": "hollow_node", "kubemark": "hollow_node",
    "local-up": "local_up", "local-up-cluster": "local_up",
    "csi-hostpath": "csi_hostpath",
    "node-problem-detector": "npd", "npd": "npd", "log-shipper": "log_shipper", "fluentd": "log_shipper",
    "gendocs": "gendocs",
    "image": "image", "kamd-image": "image", "registry": "image",
    "etcd-gateway": "etcd_gateway", "kamd-etcd-gateway": "etcd_gateway",
}


def usage():
    names = sorted({k for k in COMPONENTS if not k.startswith(("kube-", "kamd-"))})
    return "usage: hyperkube <component> [flags]\n\ncomponents:\n  " + "\n  ".join(names)


def main(argv=None):
    argv = list(sys.argv if argv is None else argv)
    prog = os.path.basename(argv[0]).replace(".py", "")
    if prog in COMPONENTS:
        comp, rest = prog, argv[1:]
    elif len(argv) > 1 and argv[1] in COMPONENTS:
        comp, rest = argv[1], argv[2:]
    else:
        print(usage(), file=sys.stderr)
        return 2
    mod = importlib.import_module(f"kubernetes_amd.cmd.{COMPONENTS[comp]}")
    sys.argv = [comp] + rest
    rc = mod.main(rest)
    return rc if isinstance(rc, int) else 0


if __name__ == "__main__":
    sys.exit(main())
