"""Node logging agent (fluentd-elasticsearch add-on equivalent) and the kubelet's
/var/log/containers symlinks it tails.

Parity: `cluster/addons/fluentd-elasticsearch/fluentd-es-configmap.yaml` (in_tail of
/var/log/containers/*.log with a pos file, docker json / CRI parsing, kubernetes_metadata filter,
elasticsearch bulk output into logstash-* indices) and `kuberuntime` legacyLogSymlink naming.
"""
import json
import os
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from kubernetes_amd.addons.logging import FileSink, ElasticsearchSink, LogShipper, parse_line, parse_name
from kubernetes_amd.addons.manager import default_addons
from kubernetes_amd.cluster import LocalCluster


class _ES:
    """Minimal Elasticsearch bulk endpoint: records every indexed document; can be 'down'."""

    def __init__(self):
        self.docs, self.down = [], False
        es = self

        class H(BaseHTTPRequestHandler):
            def do_POST(self):
                body = self.rfile.read(int(self.headers["Content-Length"])).decode()
                if es.down:
                    self.send_response(503)
                    self.end_headers()
                    return
                lines = [json.loads(x) for x in body.splitlines() if x]
                for action, doc in zip(lines[::2], lines[1::2]):
                    es.docs.append((action["index"]["_index"], doc))
                out = json.dumps({"errors": False, "items": []}).encode()
                self.send_response(200)
                self.send_header("Content-Length", str(len(out)))
                self.end_headers()
                self.wfile.write(out)

            def log_message(self, *a):
                pass
        self.srv = ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.url = f"http://127.0.0.1:{self.srv.server_address[1]}"
        threading.Thread(target=self.srv.serve_forever, daemon=True).start()

    def close(self):
        self.srv.shutdown()


def test_parsers():
    assert parse_name("/var/log/containers/gpu-job-7_ml_trainer-abc123.log") == {
        "pod": "gpu-job-7", "ns": "ml", "container": "trainer", "id": "abc123"}
    assert parse_name("junk.log") is None
    part = {}
    assert parse_line('{"log":"hello\\n","stream":"stderr","time":"2026-10-16T10:00:00Z"}', part, "k") == {
        "log": "hello\n", "stream": "stderr", "time": "2026-10-16T10:00:00Z"}
    assert parse_line("2026-10-16T10:00:00.1Z stdout P abc", part, "k") is None          # CRI partial
    assert parse_line("2026-10-16T10:00:00.2Z stdout F def", part, "k")["log"] == "abcdef\n"
    assert parse_line("plain text", part, "k")["log"] == "plain text\n"


def test_shipper_pos_file_rotation_and_retry(tmp_path, run):
    logs = tmp_path / "containers"
    logs.mkdir()
    target = tmp_path / "c1.log"
    target.write_text("old line before the agent started\n")
    link = logs / "web-0_default_app-c1.log"
    os.symlink(target, link)
    es = _ES()

    async def main():
        sh = LogShipper(str(logs), ElasticsearchSink(es.url), None, str(tmp_path / "pos"), "node-a").start()
        sh._task.cancel()
        with open(target, "a") as f:
            f.write("first\nsecond\npartial")
        await sh.run_once()
        got = [d["log"] for _, d in es.docs]
        assert got == ["first\n", "second\n"]                      # backlog skipped, partial held back
        idx, doc = es.docs[0]
        assert idx.startswith("logstash-") and doc["kubernetes"]["pod_name"] == "web-0"
        assert doc["kubernetes"]["container_name"] == "app" and doc["docker"]["container_id"] == "c1"
        # sink down: records stay buffered, then go out after the back-off
        es.down = True
        with open(target, "a") as f:
            f.write(" done\n")
        await sh.run_once()
        assert len(es.docs) == 2 and len(sh.buffer) == 1
        es.down = False
        sh._retry_at = 0
        await sh.run_once()
        assert es.docs[-1][1]["log"] == "partial done\n"
        # rotation: the file is replaced (new inode) -> read from the start
        os.unlink(target)
        target.write_text("after rotation\n")
        await sh.run_once()
        assert es.docs[-1][1]["log"] == "after rotation\n"
        await sh.stop()
        # a restarted agent resumes from the pos file: nothing is shipped twice
        n = len(es.docs)
        sh2 = LogShipper(str(logs), ElasticsearchSink(es.url), None, str(tmp_path / "pos"), "node-a").start()
        sh2._task.cancel()
        await sh2.run_once()
        assert len(es.docs) == n
        with open(target, "a") as f:
            f.write("resumed\n")
        await sh2.run_once()
        assert es.docs[-1][1]["log"] == "resumed\n" and len(es.docs) == n + 1
        await sh2.stop()
    try:
        run(main())
    finally:
        es.close()


def test_kubelet_log_symlinks_feed_the_shipper(tmp_path, run):
    """A pod on a process-runtime node writes to stdout; the kubelet's /var/log/containers
    symlink exposes it and the agent ships it with pod labels and host from the API."""
    logdir = tmp_path / "containers"
    out = tmp_path / "shipped.jsonl"

    async def main():
        cl = LocalCluster(nodes=1, gpus_per_node=0, runtime="process", workdir=str(tmp_path / "c"),
                          kubelet_kwargs={"container_log_dir": str(logdir)})
        await cl.start()
        c = cl.client
        sh = LogShipper(str(logdir), FileSink(str(out)), c, None, cl.nodes[0].name, period=0.05).start()
        try:
            await c.create("pods", {"metadata": {"name": "talker", "labels": {"app": "hip"}},
                                    "spec": {"containers": [{"name": "main", "image": "busybox",
                                                             "command": ["sh", "-c", "echo hello-from-gfx950; sleep 30"]}]}},
                           "default")

            async def shipped():
                if not out.exists():
                    return None
                recs = [json.loads(x) for x in out.read_text().splitlines()]
                return [r for r in recs if "hello-from-gfx950" in r["log"]] or None
            recs = await cl.wait_for(shipped, 20)
            k = recs[0]["kubernetes"]
            assert k["pod_name"] == "talker" and k["namespace_name"] == "default" and k["container_name"] == "main"
            assert k["labels"] == {"app": "hip"} and k["host"] == cl.nodes[0].name and k["pod_id"]
            links = os.listdir(logdir)
            assert len(links) == 1 and links[0].startswith("talker_default_main-")
            await c.delete("pods", "talker", "default", grace_period=0)

            async def unlinked():
                return not os.listdir(logdir)
            await cl.wait_for(unlinked, 20)
        finally:
            await sh.stop()
            await cl.stop()
    run(main(), timeout=90)


def test_addon_manifests_include_logging_and_default_storage_class():
    objs = {o["metadata"]["name"]: o for o in default_addons()}
    ds = objs["log-shipper"]
    cmd = ds["spec"]["template"]["spec"]["containers"][0]["command"]
    assert "kubernetes_amd.cmd.log_shipper" in cmd and "--elasticsearch" in cmd
    sc = objs["standard"]
    assert sc["kind"] == "StorageClass" and sc["metadata"]["annotations"]["storageclass.beta.kubernetes.io/is-default-class"] == "true"
