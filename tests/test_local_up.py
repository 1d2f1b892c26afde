"""Multi-process cluster (hack/local-up-cluster.sh equivalent): every component in its own
process, talking over HTTP and gRPC/unix sockets; kubectl drives it."""
import io
import os
import signal
import subprocess
import sys
import time

import pytest

from kubernetes_amd.kubectl.cli import main as kubectl

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def local_up(tmp_path_factory):
    wd = str(tmp_path_factory.mktemp("localup"))
    ready = os.path.join(wd, "ready")
    env = dict(os.environ, PYTHONPATH=ROOT)
    p = subprocess.Popen([sys.executable, "-m", "kubernetes_amd.cmd.local_up", "--workdir", wd, "--fake-gpus", "8",
                          "--runtime", "stub", "--node-name", "mi355x-local", "--ready-file", ready, "--exporter-port", "0"],
                         env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, start_new_session=True)
    t = time.time()
    while not os.path.exists(ready):
        if p.poll() is not None or time.time() - t > 90:
            out = p.stdout.read().decode() if p.poll() is not None else ""
            raise RuntimeError("local-up failed " + out)
        time.sleep(0.1)
    yield open(ready).read(), wd
    os.killpg(p.pid, signal.SIGTERM)
    p.wait(30)


def k(url, *args):
    out = io.StringIO()
    rc = kubectl(["-s", url] + list(args), out=out)
    return rc, out.getvalue()


def wait(pred, timeout=60):
    t = time.time()
    while time.time() - t < timeout:
        r = pred()
        if r:
            return r
        time.sleep(0.2)
    raise TimeoutError


def test_node_registers_gpus_across_processes(local_up):
    url, _ = local_up
    wait(lambda: "8/8" in k(url, "get", "nodes")[1])
    rc, out = k(url, "get", "nodes", "-o", "wide")
    assert "mi355x-local" in out and "MI355X" in out


def test_gpu_pod_through_separate_processes(local_up):
    url, _ = local_up
    wait(lambda: "8/8" in k(url, "get", "nodes")[1])
    rc, out = k(url, "run", "gpujob", "--image", "kubernetes-amd/hip-vector-add", "--gpus", "2", "--restart", "Never")
    assert rc == 0
    wait(lambda: "Running" in k(url, "get", "pod", "gpujob")[1])
    rc, out = k(url, "describe", "pod", "gpujob")
    assert out.count("GPU-") >= 2
