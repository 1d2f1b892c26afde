"""local-up-cluster: every component as its own process on this machine (reference:
hack/local-up-cluster.sh, 943 lines of shell). kube-apiserver, kube-controller-manager,
kube-scheduler, kubelet and the amd.com/gpu device plugin (real AMD SMI, or a fake N x MI355X
fixture with --fake-gpus), plus a kubeconfig for kubectl.

    python -m kubernetes_amd.cmd.local_up --workdir /tmp/kamd --fake-gpus 8
"""
from __future__ import annotations

import argparse
import os
import signal
import subprocess
import sys
import time

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def spawn(args, log, env):
    return subprocess.Popen([sys.executable, "-m"] + args, stdout=open(log, "w"), stderr=subprocess.STDOUT, env=env,
                            start_new_session=True)


def main(argv=None):
    ap = argparse.ArgumentParser("local-up-cluster")
    ap.add_argument("--workdir", default="/tmp/kubernetes-amd")
    ap.add_argument("--fake-gpus", type=int, default=0, help="0 = use the real GPUs through AMD SMI")
    ap.add_argument("--runtime", default="process", choices=["process", "stub"])
    ap.add_argument("--node-name", default=os.uname().nodename)
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--no-controllers", action="store_true")
    ap.add_argument("--exporter-port", type=int, default=None)
    ap.add_argument("--ready-file", default=None)
    a = ap.parse_args(argv)
    os.makedirs(a.workdir, exist_ok=True)
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    procs = []
    pf = os.path.join(a.workdir, "apiserver.port")
    if os.path.exists(pf):
        os.unlink(pf)
    try:
        procs.append(spawn(["kubernetes_amd.cmd.apiserver", "--port", str(a.port), "--port-file", pf,
                            "--etcd-wal", os.path.join(a.workdir, "etcd.wal")], os.path.join(a.workdir, "apiserver.log"), env))
        t = time.time()
        while not os.path.exists(pf):
            if procs[0].poll() is not None or time.time() - t > 60:
                raise SystemExit("apiserver failed: see " + os.path.join(a.workdir, "apiserver.log"))
            time.sleep(0.05)
        url = f"http://127.0.0.1:{open(pf).read().strip()}"
        procs.append(spawn(["kubernetes_amd.cmd.scheduler", "--master", url], os.path.join(a.workdir, "scheduler.log"), env))
        if not a.no_controllers:
            procs.append(spawn(["kubernetes_amd.cmd.controller_manager", "--master", url],
                               os.path.join(a.workdir, "controller-manager.log"), env))
        pdir = os.path.join(a.workdir, "kubelet", "device-plugin", "plugins")
        procs.append(spawn(["kubernetes_amd.cmd.kubelet", "--master", url, "--hostname-override", a.node_name,
                            "--root-dir", os.path.join(a.workdir, "kubelet"), "--device-plugins-dir", pdir,
                            "--container-runtime", a.runtime, "--port", "0"], os.path.join(a.workdir, "kubelet.log"), env))
        dp = ["kubernetes_amd.cmd.device_plugin", "--plugins-dir", pdir, "--node-name", a.node_name]
        if a.fake_gpus:
            dp += ["--fake-gpus", str(a.fake_gpus)]
        if a.exporter_port is not None:
            dp += ["--exporter-port", str(a.exporter_port)]
        procs.append(spawn(dp, os.path.join(a.workdir, "device-plugin.log"), env))
        kc = os.path.join(a.workdir, "kubeconfig")
        with open(kc, "w") as f:
            yaml.safe_dump({"apiVersion": "v1", "kind": "Config", "current-context": "local",
                            "clusters": [{"name": "local", "cluster": {"server": url}}],
                            "users": [{"name": "admin", "user": {}}],
                            "contexts": [{"name": "local", "context": {"cluster": "local", "user": "admin", "namespace": "default"}}]}, f)
        print(f"Local cluster is running. API server: {url}\n  export KUBECONFIG={kc}\n"
              f"  python -m kubernetes_amd.kubectl get nodes -o wide\nLogs in {a.workdir}", flush=True)
        if a.ready_file:
            with open(a.ready_file, "w") as f:
                f.write(url)
        stop = []
        signal.signal(signal.SIGTERM, lambda *_: stop.append(1))
        signal.signal(signal.SIGINT, lambda *_: stop.append(1))
        while not stop:
            for p in procs:
                if p.poll() is not None:
                    print(f"component {p.args[3]} exited with {p.returncode}", flush=True)
                    stop.append(1)
            time.sleep(0.2)
    finally:
        for p in reversed(procs):
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                p.kill()


if __name__ == "__main__":
    main()
