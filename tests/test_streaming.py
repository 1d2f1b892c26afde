"""kubectl exec / attach / port-forward / cp / proxy / edit through the API server and kubelet
streaming endpoints, for an in-process runtime and for a CRI (gRPC) runtime.

Parity: `test/e2e/kubectl/kubectl.go` ("should support exec", "should support port-forward"),
`pkg/kubelet/server/server_test.go` (exec/portForward routes).
"""
import asyncio
import io
import os
import socket
import sys

import pytest

from kubernetes_amd.cluster import LocalCluster
from kubernetes_amd.cri.remote import RemoteRuntime
from kubernetes_amd.cri.server import CRIServer
from kubernetes_amd.kubectl.cli import Kubectl, build_parser
from kubernetes_amd.kubelet.runtime.process import ProcessRuntime


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


ECHO = ("import socket,sys\n"
        "s=socket.socket(); s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)\n"
        "s.bind(('127.0.0.1', int(sys.argv[1]))); s.listen(8); print('listening', flush=True)\n"
        "while True:\n"
        "    c,_=s.accept(); d=c.recv(100); c.sendall(b'pong:'+d); c.close(); print('served', d.decode(), flush=True)\n")


def kubectl(url, *argv):
    out = io.StringIO()
    k = Kubectl(build_parser().parse_args(["-s", url, *argv]), out)
    k.rc = 0
    return k, out


async def _scenario(cl, node_name=None):
    port = free_port()
    await cl.client.create("pods", {"metadata": {"name": "srv", "namespace": "default"},
                                    "spec": {"nodeName": node_name or cl.nodes[0].name, "containers": [
                                        {"name": "main", "image": "busybox", "command": [sys.executable, "-c", ECHO, str(port)]}]}})
    await cl.wait_pod("srv")
    # wait until the echo server is up (log line)
    for _ in range(200):
        k, out = kubectl(cl.url, "logs", "srv")
        await k.cmd_logs()
        await k.client.close()
        if "listening" in out.getvalue():
            break
        await asyncio.sleep(0.05)
    k, out = kubectl(cl.url, "exec", "srv", "--", "sh", "-c", "echo hi-from-exec; exit 4")
    await k.cmd_exec()
    await k.client.close()
    assert out.getvalue() == "hi-from-exec\n" and k.rc == 4
    k, out = kubectl(cl.url, "exec", "srv", "-c", "nope", "--", "true")
    with pytest.raises(SystemExit):
        await k.cmd_exec()
    await k.client.close()
    # port-forward: one tunnelled connection, then the command returns
    k, out = kubectl(cl.url, "port-forward", "pod/srv", f"0:{port}", "--max-connections", "1")
    task = asyncio.ensure_future(k.cmd_port_forward())
    for _ in range(100):
        if "Forwarding from" in out.getvalue():
            break
        await asyncio.sleep(0.02)
    local = int(out.getvalue().split("Forwarding from 127.0.0.1:")[1].split()[0])
    r, w = await asyncio.open_connection("127.0.0.1", local)
    w.write(b"ping")
    await w.drain()
    assert await asyncio.wait_for(r.read(100), 10) == b"pong:ping"
    w.close()
    await asyncio.wait_for(task, 10)
    await k.client.close()
    return port


def test_exec_portforward_cp_inprocess(run, tmp_path):
    async def main():
        cl = LocalCluster(nodes=1, gpus_per_node=0, runtime="process", kubelet_http=True, workdir=str(tmp_path / "c"))
        await cl.start()
        try:
            port = await _scenario(cl)
            # cp both ways
            src = tmp_path / "local.txt"
            src.write_bytes(b"payload \x00\x01 'quoted'\n")
            k, _ = kubectl(cl.url, "cp", str(src), f"srv:{tmp_path}/in-pod.bin")
            await k.cmd_cp()
            await k.client.close()
            assert (tmp_path / "in-pod.bin").read_bytes() == src.read_bytes()
            k, _ = kubectl(cl.url, "cp", f"srv:{tmp_path}/in-pod.bin", str(tmp_path / "back.bin"))
            await k.cmd_cp()
            await k.client.close()
            assert (tmp_path / "back.bin").read_bytes() == src.read_bytes()
            # directories and files past the old 1 MiB limit travel as tar streams
            tree = tmp_path / "tree"
            (tree / "sub").mkdir(parents=True)
            big = os.urandom(3 << 20)
            (tree / "sub" / "big.bin").write_bytes(big)
            (tree / "a.txt").write_text("A")
            k, _ = kubectl(cl.url, "cp", str(tree), f"srv:{tmp_path}/pod-tree")
            await k.cmd_cp()
            await k.client.close()
            assert (tmp_path / "pod-tree" / "sub" / "big.bin").read_bytes() == big
            k, _ = kubectl(cl.url, "cp", f"default/srv:{tmp_path}/pod-tree", str(tmp_path / "tree-back"))
            await k.cmd_cp()
            await k.client.close()
            assert (tmp_path / "tree-back" / "a.txt").read_text() == "A"
            assert (tmp_path / "tree-back" / "sub" / "big.bin").read_bytes() == big
            # attach streams what the running container writes from now on
            k, out = kubectl(cl.url, "attach", "srv")
            task = asyncio.ensure_future(k.cmd_attach())
            await asyncio.sleep(0.5)
            r, w = await asyncio.open_connection("127.0.0.1", port)
            w.write(b"live")
            await w.drain()
            assert await asyncio.wait_for(r.read(100), 10) == b"pong:live"
            w.close()
            for _ in range(200):
                if "served live" in out.getvalue():
                    break
                await asyncio.sleep(0.02)
            assert "served live" in out.getvalue() and "listening" not in out.getvalue()
            task.cancel()
            await k.client.close()
        finally:
            await cl.stop()
    run(main(), timeout=90)


def test_exec_portforward_over_cri(run, tmp_path):
    async def main():
        sock = str(tmp_path / "cri.sock")
        prt = ProcessRuntime(str(tmp_path / "rt"))
        srv = await CRIServer(prt, sock).start()
        rt = await RemoteRuntime(sock, relist_period=0.1).connect()
        cl = LocalCluster(nodes=0, gpus_per_node=0, kubelet_http=True, workdir=str(tmp_path / "c"))
        await cl.start()
        try:
            await cl.add_node("cri-node", runtime=rt)
            await _scenario(cl, "cri-node")
        finally:
            await cl.stop()
            await rt.close()
            await srv.stop()
            await prt.kill_all()     # containers outlive a CRI server stop by design
    run(main(), timeout=90)


def test_proxy_and_edit(run, tmp_path):
    async def main():
        cl = LocalCluster(nodes=0, gpus_per_node=0)
        await cl.start()
        try:
            await cl.client.create("configmaps", {"metadata": {"name": "cm", "namespace": "default"}, "data": {"k": "v1"}})
            port = free_port()
            k, out = kubectl(cl.url, "proxy", "--port", str(port), "--serve-seconds", "3")
            task = asyncio.ensure_future(k.cmd_proxy())
            for _ in range(100):
                if "Starting to serve" in out.getvalue():
                    break
                await asyncio.sleep(0.02)
            from kubernetes_amd.client.rest import Client
            c = Client(f"http://127.0.0.1:{port}")
            assert (await c.get("configmaps", "cm", "default"))["data"] == {"k": "v1"}
            await c.close()
            task.cancel()
            await k.client.close()
            editor = tmp_path / "ed.sh"
            editor.write_text("#!/bin/sh\nsed -i 's/k: v1/k: v2/' \"$1\"\n")
            os.chmod(editor, 0o755)
            os.environ["KUBE_EDITOR"] = str(editor)
            try:
                k, out = kubectl(cl.url, "edit", "configmap/cm")
                await k.cmd_edit()
                await k.client.close()
            finally:
                os.environ.pop("KUBE_EDITOR", None)
            assert "configmap/cm edited" in out.getvalue()
            assert (await cl.client.get("configmaps", "cm", "default"))["data"] == {"k": "v2"}
        finally:
            await cl.stop()
    run(main(), timeout=60)
