"""Node logging agent: ships container logs with Kubernetes metadata to Elasticsearch.

Parity: the `cluster/addons/fluentd-elasticsearch` add-on (a fluentd DaemonSet,
`fluentd-es-configmap.yaml` `containers.input.conf` + `output.conf`). Its behaviour is kept:
  * **input**: tail `/var/log/containers/*.log` — the kubelet's
    `<pod>_<namespace>_<container>-<containerID>.log` symlinks — from the end for new files
    (`read_from_head false`), with positions persisted in a pos file so a restarted agent
    resumes where it left off, and rotation/truncation detected by inode and size;
  * **parsing**: Docker json-file lines (`{"log", "stream", "time"}`), CRI lines
    (`<time> <stream> <F|P> <msg>`, partial lines joined) or plain text;
  * **kubernetes_metadata filter**: namespace, pod name/uid, container name/id from the file
    name, plus pod labels and host from the API (cached per pod);
  * **output**: the Elasticsearch bulk API into daily `logstash-YYYY.MM.DD` indices (buffered,
    retried with back-off when the sink is down, batches bounded), or a JSON-lines file / stdout.
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import re
import time
from datetime import datetime, timezone

from ..client.rest import APIStatusError

log = logging.getLogger("log-shipper")

NAME_RE = re.compile(r"^(?P<pod>[a-z0-9]([-a-z0-9.]*[a-z0-9])?)_(?P<ns>[^_]+)_(?P<container>.+)-(?P<id>[^-]+)\.log$")
CRI_RE = re.compile(r"^(?P<time>\S+) (?P<stream>stdout|stderr) (?P<tag>[FP]) (?P<log>.*)$")


def parse_name(fname):
    m = NAME_RE.match(os.path.basename(fname))
    return m.groupdict() if m else None


def parse_line(line: str, partial: dict, key):
    """-> record dict or None (a CRI partial line kept for the next one)."""
    line = line.rstrip("\n")
    if line.startswith("{"):
        try:
            d = json.loads(line)
            if isinstance(d, dict) and "log" in d:
                return {"log": d["log"], "stream": d.get("stream", "stdout"), "time": d.get("time")}
        except ValueError:
            pass
    m = CRI_RE.match(line)
    if m:
        if m["tag"] == "P":
            partial[key] = partial.get(key, "") + m["log"]
            return None
        return {"log": partial.pop(key, "") + m["log"] + "\n", "stream": m["stream"], "time": m["time"]}
    return {"log": line + "\n", "stream": "stdout", "time": None}


class PosFile:
    """`pos_file`: path -> (inode, offset), written atomically."""

    def __init__(self, path):
        self.path = path
        self.pos: dict[str, list] = {}
        if path and os.path.exists(path):
            try:
                with open(path) as f:
                    self.pos = json.load(f)
            except (OSError, ValueError):
                self.pos = {}

    def save(self):
        if not self.path:
            return
        tmp = self.path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(self.pos, f)
        os.replace(tmp, self.path)


class ElasticsearchSink:
    """Bulk API: one `index` action per record into logstash-YYYY.MM.DD."""

    def __init__(self, url, index_prefix="logstash", timeout=10.0):
        self.url = url.rstrip("/")
        self.prefix = index_prefix
        self.timeout = timeout

    def _post(self, url, body, headers):
        import urllib.error
        import urllib.request
        req = urllib.request.Request(url, data=body, headers=headers, method="POST")
        try:
            with urllib.request.urlopen(req, timeout=self.timeout) as r:
                return r.status, r.read()
        except urllib.error.HTTPError as e:
            return e.code, e.read()

    async def send(self, records):
        lines = []
        for r in records:
            day = r["@timestamp"][:10].replace("-", ".")
            lines.append(json.dumps({"index": {"_index": f"{self.prefix}-{day}", "_type": "fluentd"}}))
            lines.append(json.dumps(r, separators=(",", ":")))
        body = ("\n".join(lines) + "\n").encode()
        loop = asyncio.get_running_loop()
        status, resp = await loop.run_in_executor(None, self._post, self.url + "/_bulk", body,
                                                  {"Content-Type": "application/x-ndjson"})
        if status >= 300:
            raise OSError(f"bulk request failed: HTTP {status}: {resp[:200]!r}")
        d = json.loads(resp or b"{}")
        if d.get("errors"):
            raise OSError("bulk request had item errors")


class FileSink:
    def __init__(self, path):
        self.path = path

    async def send(self, records):
        if self.path == "-":
            for r in records:
                print(json.dumps(r), flush=True)
            return
        with open(self.path, "a") as f:
            for r in records:
                f.write(json.dumps(r, separators=(",", ":")) + "\n")


class LogShipper:
    def __init__(self, log_dir, sink, client=None, pos_file=None, node_name="", period=1.0, batch=1000,
                 max_buffer=100_000, read_from_head=False):
        self.log_dir = log_dir
        self.sink = sink
        self.client = client
        self.pos = PosFile(pos_file)
        self.node = node_name
        self.period = period
        self.batch = batch
        self.max_buffer = max_buffer
        self.read_from_head = read_from_head
        self.buffer: list = []
        self.dropped = 0
        self.shipped = 0
        self._partial: dict = {}
        self._meta: dict = {}
        self._task = None
        self._backoff = 0.0
        self._retry_at = 0.0

    # -- input -------------------------------------------------------------
    def _files(self):
        try:
            names = os.listdir(self.log_dir)
        except OSError:
            return []
        return [os.path.join(self.log_dir, n) for n in sorted(names) if n.endswith(".log")]

    def _read_new(self, path):
        try:
            st = os.stat(path)                        # follows the symlink to the runtime's file
        except OSError:
            return []
        ino, size = st.st_ino, st.st_size
        ent = self.pos.pos.get(path)
        if ent is None:
            off = 0          # a log that appeared while we run is read from its start
        else:
            old_ino, off = ent
            if old_ino != ino or size < off:          # rotated or truncated: start over
                off = 0
        if size == off:
            self.pos.pos[path] = [ino, off]
            return []
        with open(path, "rb") as f:
            f.seek(off)
            data = f.read(size - off)
        cut = data.rfind(b"\n") + 1
        self.pos.pos[path] = [ino, off + cut]
        return data[:cut].decode(errors="replace").splitlines()

    async def _metadata(self, ns, pod):
        key = (ns, pod)
        if key in self._meta:
            return self._meta[key]
        meta = {}
        if self.client is not None:
            try:
                p = await self.client.get("pods", pod, ns)
                md = p["metadata"]
                meta = {"pod_id": md.get("uid"), "labels": md.get("labels") or {},
                        "host": (p.get("spec") or {}).get("nodeName") or self.node}
            except (APIStatusError, OSError, ConnectionError):
                meta = {}
        self._meta[key] = meta
        return meta

    async def collect_once(self):
        live = set()
        for path in self._files():
            live.add(path)
            info = parse_name(path)
            lines = self._read_new(path)
            if not lines or info is None:
                continue
            meta = await self._metadata(info["ns"], info["pod"])
            for ln in lines:
                rec = parse_line(ln, self._partial, path)
                if rec is None:
                    continue
                ts = rec.pop("time") or datetime.now(timezone.utc).isoformat().replace("+00:00", "Z")
                rec["@timestamp"] = ts
                rec["kubernetes"] = {"namespace_name": info["ns"], "pod_name": info["pod"],
                                     "container_name": info["container"], "host": meta.get("host", self.node),
                                     **({"pod_id": meta["pod_id"]} if meta.get("pod_id") else {}),
                                     **({"labels": meta["labels"]} if meta.get("labels") else {})}
                rec["docker"] = {"container_id": info["id"]}
                self.buffer.append(rec)
        for gone in set(self.pos.pos) - live:          # deleted logs: forget their positions
            del self.pos.pos[gone]
        if len(self.buffer) > self.max_buffer:          # buffer overflow: drop the oldest
            self.dropped += len(self.buffer) - self.max_buffer
            del self.buffer[:len(self.buffer) - self.max_buffer]

    # -- output ------------------------------------------------------------
    async def flush_once(self):
        if not self.buffer or time.monotonic() < self._retry_at:
            return
        while self.buffer:
            chunk = self.buffer[:self.batch]
            try:
                await self.sink.send(chunk)
            except (OSError, ConnectionError, ValueError) as e:
                self._backoff = min(max(self._backoff * 2, 0.5), 30.0)
                self._retry_at = time.monotonic() + self._backoff
                log.warning("log sink unavailable (%s); retrying in %.1fs, %d records buffered", e, self._backoff,
                            len(self.buffer))
                return
            del self.buffer[:len(chunk)]
            self.shipped += len(chunk)
            self._backoff = 0.0
        self.pos.save()

    async def run_once(self):
        await self.collect_once()
        await self.flush_once()

    async def _loop(self):
        while True:
            try:
                await self.run_once()
            except Exception as e:  # noqa: BLE001 - the agent keeps going
                log.warning("log shipping pass failed: %s", e)
            await asyncio.sleep(self.period)

    def start(self):
        if not self.read_from_head:
            for p in self._files():       # content already there at start is skipped (read_from_head false)
                if p not in self.pos.pos:
                    try:
                        st = os.stat(p)
                        self.pos.pos[p] = [st.st_ino, st.st_size]
                    except OSError:
                        pass
        self._task = asyncio.ensure_future(self._loop())
        return self

    async def stop(self):
        if self._task:
            self._task.cancel()
            try:
                await self._task
            except asyncio.CancelledError:
                pass
        await self.flush_once()
        self.pos.save()


def main(argv=None):
    import argparse
    import sys

    from ..client.rest import Client
    from .npd import apiserver_url
    ap = argparse.ArgumentParser("log-shipper")
    ap.add_argument("--log-dir", default="/var/log/containers")
    ap.add_argument("--pos-file", default="/var/log/es-containers.log.pos")
    ap.add_argument("--elasticsearch", default=None, help="Elasticsearch URL (bulk API); default: --output")
    ap.add_argument("--output", default="-", help="JSON-lines file when no Elasticsearch is given ('-' = stdout)")
    ap.add_argument("--master", default=None)
    ap.add_argument("--node-name", default=os.environ.get("NODE_NAME") or os.uname().nodename)
    ap.add_argument("--period", type=float, default=1.0)
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, stream=sys.stderr)
    sink = ElasticsearchSink(a.elasticsearch) if a.elasticsearch else FileSink(a.output)

    async def run():
        client = Client(apiserver_url(a.master))
        sh = LogShipper(a.log_dir, sink, client, a.pos_file, a.node_name, a.period).start()
        try:
            await asyncio.Event().wait()
        finally:
            await sh.stop()
            await client.close()
    asyncio.run(run())


if __name__ == "__main__":
    main()
