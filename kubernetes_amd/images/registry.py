"""Docker Registry HTTP API v2 client (pull): what the dockershim's docker daemon does for
`PullImage` (`pkg/kubelet/dockershim/docker_image.go:PullImage` with the kubelet's credentials
from `pkg/credentialprovider` keyrings).

  * `GET /v2/<name>/manifests/<tag|digest>` with the OCI / Docker v2 manifest and index media
    types; an index (manifest list) selects the `linux/<arch>` entry;
  * `GET /v2/<name>/blobs/<digest>` for the config and layers, streamed to the store with
    digest verification, following redirects (blob storage backends);
  * auth: a 401 `WWW-Authenticate: Bearer realm=…,service=…,scope=…` challenge is answered by
    fetching a token from the realm (HTTP basic with the pull credentials when there are any),
    `Basic` challenges get the credentials directly;
  * plain HTTP for `localhost`/`127.0.0.0/8` registries and those listed as insecure (docker's
    `--insecure-registry`), HTTPS with certificate verification for the rest.
"""
from __future__ import annotations

import asyncio
import base64
import ipaddress
import json
import platform
import re
import ssl
from urllib.parse import urlencode, urljoin, urlsplit

from . import reference
from .store import INDEX_TYPES, MANIFEST_TYPES, OCIStore

ACCEPT = ", ".join(MANIFEST_TYPES + INDEX_TYPES)
ARCH = {"x86_64": "amd64", "aarch64": "arm64"}.get(platform.machine(), platform.machine())


class RegistryError(Exception):
    def __init__(self, status, message):
        super().__init__(f"{message} (HTTP {status})" if status else message)
        self.status = status


class Auth:
    """Pull credentials for one registry (CRI AuthConfig)."""

    def __init__(self, username="", password="", auth="", identity_token="", registry_token=""):
        if auth and not username:
            try:
                username, _, password = base64.b64decode(auth).decode().partition(":")
            except (ValueError, UnicodeDecodeError):
                pass
        self.username, self.password = username, password
        self.identity_token, self.registry_token = identity_token, registry_token

    def basic(self) -> str | None:
        if not self.username:
            return None
        return "Basic " + base64.b64encode(f"{self.username}:{self.password}".encode()).decode()


async def _fetch(url, headers, sink=None, insecure=False, max_redirects=5, timeout=300.0):
    """-> (status, headers, body). With `sink`, a 200 body is streamed into sink.write()."""
    for _ in range(max_redirects + 1):
        u = urlsplit(url)
        port = u.port or (443 if u.scheme == "https" else 80)
        ctx = None
        if u.scheme == "https":
            ctx = ssl.create_default_context()
            if insecure:
                ctx.check_hostname = False
                ctx.verify_mode = ssl.CERT_NONE
        r, w = await asyncio.wait_for(asyncio.open_connection(u.hostname, port, ssl=ctx, limit=1 << 22), 30)
        try:
            target = (u.path or "/") + ("?" + u.query if u.query else "")
            lines = [f"GET {target} HTTP/1.1", f"Host: {u.hostname}:{port}", "Connection: close",
                     "User-Agent: kamd-kubelet/1.9"] + [f"{k}: {v}" for k, v in headers.items()]
            w.write(("\r\n".join(lines) + "\r\n\r\n").encode())
            await w.drain()
            head = await asyncio.wait_for(r.readuntil(b"\r\n\r\n"), timeout)
            status_line, _, rest = head.decode("latin-1").partition("\r\n")
            status = int(status_line.split(" ", 2)[1])
            hdrs = {}
            for ln in rest.split("\r\n"):
                k, _, v = ln.partition(":")
                if k:
                    hdrs[k.strip().lower()] = v.strip()
            if status in (301, 302, 303, 307, 308) and "location" in hdrs:
                url = urljoin(url, hdrs["location"])
                if urlsplit(url).netloc != u.netloc:
                    headers = {k: v for k, v in headers.items() if k.lower() != "authorization"}
                continue
            out = bytearray() if (sink is None or status != 200) else None

            def emit(d):
                if out is not None:
                    out.extend(d)
                else:
                    sink.write(d)
            if hdrs.get("transfer-encoding", "").lower() == "chunked":
                while True:
                    n = int((await r.readline()).strip().split(b";")[0], 16)
                    if n == 0:
                        break
                    emit(await asyncio.wait_for(r.readexactly(n), timeout))
                    await r.readline()
            elif "content-length" in hdrs:
                left = int(hdrs["content-length"])
                while left:
                    d = await asyncio.wait_for(r.read(min(left, 1 << 20)), timeout)
                    if not d:
                        raise RegistryError(status, "connection closed mid-body")
                    emit(d)
                    left -= len(d)
            else:
                while True:
                    d = await asyncio.wait_for(r.read(1 << 20), timeout)
                    if not d:
                        break
                    emit(d)
            return status, hdrs, bytes(out or b"")
        finally:
            w.close()
    raise RegistryError(0, f"too many redirects fetching {url}")


def _challenge(value: str):
    scheme, _, params = value.partition(" ")
    return scheme.lower(), dict(re.findall(r'(\w+)="([^"]*)"', params))


class RegistryClient:
    def __init__(self, insecure_registries=(), timeout=300.0):
        self.insecure = set(insecure_registries)
        self.timeout = timeout
        self._tokens: dict[tuple, str] = {}

    def _scheme(self, host) -> str:
        name = host.rsplit(":", 1)[0] if host.count(":") == 1 else host
        if host in self.insecure or name == "localhost":
            return "http"
        try:
            if ipaddress.ip_address(name).is_loopback:
                return "http"
        except ValueError:
            pass
        return "https"

    async def _get(self, ref: reference.Reference, path, accept=None, sink=None, auth: Auth | None = None):
        host = ref.api_host
        url = f"{self._scheme(host)}://{host}/v2/{ref.repository}/{path}"
        headers = {"Accept": accept} if accept else {}
        key = (host, ref.repository, auth.username if auth else "")     # never share a token across credentials
        if key in self._tokens:
            headers["Authorization"] = self._tokens[key]
        st, hdrs, body = await _fetch(url, headers, sink, insecure=host in self.insecure, timeout=self.timeout)
        if st == 401 and "www-authenticate" in hdrs:
            scheme, params = _challenge(hdrs["www-authenticate"])
            if scheme == "bearer":
                self._tokens[key] = "Bearer " + await self._token(params, ref, auth)
            elif scheme == "basic" and auth and auth.basic():
                self._tokens[key] = auth.basic()
            else:
                raise RegistryError(401, f"unauthorized: authentication required for {ref.name}")
            headers["Authorization"] = self._tokens[key]
            st, hdrs, body = await _fetch(url, headers, sink, insecure=host in self.insecure, timeout=self.timeout)
        if st != 200:
            msg = body.decode(errors="replace").strip()
            try:
                errs = json.loads(body).get("errors") or []
                msg = "; ".join(f"{e.get('code')}: {e.get('message')}" for e in errs) or msg
            except (ValueError, AttributeError):
                pass
            raise RegistryError(st, f"pulling {ref}: {msg or 'request failed'}")
        return hdrs, body

    async def _token(self, params, ref, auth):
        if auth and auth.registry_token:
            return auth.registry_token
        q = {"service": params.get("service", "")}
        q["scope"] = params.get("scope") or f"repository:{ref.repository}:pull"
        headers = {}
        if auth and auth.basic():
            headers["Authorization"] = auth.basic()
        realm = params.get("realm", "")
        if not realm:
            raise RegistryError(401, "bearer challenge without a realm")
        st, _h, body = await _fetch(realm + ("&" if "?" in realm else "?") + urlencode(q), headers,
                                    insecure=urlsplit(realm).netloc in self.insecure, timeout=self.timeout)
        if st != 200:
            raise RegistryError(st, f"token request to {realm} failed: {body[:200].decode(errors='replace')}")
        tok = json.loads(body)
        return tok.get("token") or tok.get("access_token") or ""

    async def pull(self, image: str, store: OCIStore, auth: Auth | None = None) -> str:
        """Pull image into store; returns the manifest digest (the image's repo digest)."""
        ref = reference.parse(image)
        hdrs, body = await self._get(ref, f"manifests/{ref.digest or ref.tag}", ACCEPT, auth=auth)
        man = json.loads(body)
        mtype = man.get("mediaType") or hdrs.get("content-type", "").split(";")[0]
        if ref.digest:
            store.put_blob(body, ref.digest)        # verifies the pinned digest
        if mtype in INDEX_TYPES or "manifests" in man:
            chosen = None
            for m in man.get("manifests") or ():
                p = m.get("platform") or {}
                if p.get("os", "linux") == "linux" and p.get("architecture") == ARCH:
                    chosen = m
                    break
            if chosen is None:
                raise RegistryError(0, f"no linux/{ARCH} image in the index of {ref}")
            hdrs, body = await self._get(ref, f"manifests/{chosen['digest']}", ACCEPT, auth=auth)
            store.put_blob(body, chosen["digest"])
            man = json.loads(body)
        if man.get("schemaVersion") != 2 or "config" not in man:
            raise RegistryError(0, f"unsupported manifest for {ref} (schema 1 images are not supported)")
        md = store.put_blob(body)
        for desc in [man["config"]] + list(man.get("layers") or ()):
            d = desc["digest"]
            if store.has_blob(d):
                continue
            wr = store.blob_writer(d)
            try:
                await self._get(ref, f"blobs/{d}", sink=wr, auth=auth)
                wr.commit()
            except BaseException:
                wr.abort()
                raise
        store.tag(str(ref), md)        # tag, or `name@digest` for a pinned pull (an index digest maps here)
        return md
