"""A read-only Docker Registry HTTP API v2 server over a node-local OCIStore — the cluster's
in-cluster registry add-on (`cluster/addons/registry` in the reference runs the upstream
registry image behind `kube-registry-proxy`) for air-gapped MI355X clusters, and the registry
the image tests pull from.

Routes: `GET /v2/` (API version check), `GET|HEAD /v2/<name>/manifests/<tag|digest>` (with
`Docker-Content-Digest`), `GET|HEAD /v2/<name>/blobs/<digest>`, `GET /v2/_catalog`,
`GET /v2/<name>/tags/list`. With `users`, requests need a bearer token from `GET /token`
(HTTP basic), answered by the standard `WWW-Authenticate: Bearer realm=…` challenge.
"""
from __future__ import annotations

import base64
import json
import secrets

from ..utils.httpserver import HTTPServer, Response
from . import reference
from .store import OCIStore


def _err(status, code, msg, headers=None):
    body = json.dumps({"errors": [{"code": code, "message": msg}]}).encode()
    return Response(status, body, "application/json", dict(headers or {}, **{"Docker-Distribution-API-Version": "registry/2.0"}))


class RegistryServer:
    def __init__(self, store: OCIStore, host="127.0.0.1", users: dict | None = None):
        self.store, self.host, self.users = store, host, users
        self.tokens: set[str] = set()
        self.http = HTTPServer(self.handle)
        self.port = None
        self.requests = 0

    async def start(self, port=0):
        self.port = await self.http.start(self.host, port)
        return self

    async def stop(self):
        await self.http.stop()

    @property
    def address(self):
        return f"{self.host}:{self.port}"

    def _authorized(self, req):
        if not self.users:
            return True
        a = req.headers.get("authorization", "")
        return a.startswith("Bearer ") and a[7:] in self.tokens

    def _challenge(self, name):
        realm = f"http://{self.address}/token"
        return _err(401, "UNAUTHORIZED", "authentication required", {
            "WWW-Authenticate": f'Bearer realm="{realm}",service="kamd-registry",scope="repository:{name}:pull"'})

    async def handle(self, req):
        self.requests += 1
        path = req.path
        if path == "/token":
            a = req.headers.get("authorization", "")
            try:
                user, _, pw = base64.b64decode(a[6:]).decode().partition(":") if a.startswith("Basic ") else ("", "", "")
            except (ValueError, UnicodeDecodeError):
                user, pw = "", ""
            if not self.users or self.users.get(user) != pw:
                return _err(401, "UNAUTHORIZED", "bad credentials")
            tok = secrets.token_urlsafe(16)
            self.tokens.add(tok)
            return Response(200, json.dumps({"token": tok}).encode())
        if not path.startswith("/v2/"):
            return _err(404, "NOT_FOUND", "not found")
        if path == "/v2/":
            return self._challenge("") if not self._authorized(req) else Response(200, b"{}")
        if path == "/v2/_catalog":
            repos = sorted({reference.parse(t).repository for t in self.store.repos})
            return Response(200, json.dumps({"repositories": repos}).encode())
        rest = path[4:]
        for kind in ("/manifests/", "/blobs/", "/tags/list"):
            i = rest.rfind(kind)
            if i > 0:
                name, arg = rest[:i], rest[i + len(kind):]
                break
        else:
            return _err(404, "NOT_FOUND", "unknown route")
        if not self._authorized(req):
            return self._challenge(name)
        full = f"{self.address}/{name}"
        if kind == "/tags/list":
            tags = sorted(reference.parse(t).tag for t in self.store.repos
                          if reference.parse(t).repository == name and reference.parse(t).tag)
            return Response(200, json.dumps({"name": name, "tags": tags}).encode())
        if kind == "/manifests/":
            md = self.store.resolve(f"{full}@{arg}" if arg.startswith("sha256:") else f"{full}:{arg}")
            if md is None:
                # images are stored under whatever name they were tagged with: also match by repository
                for t, d in self.store.repos.items():
                    r = reference.parse(t)
                    if r.repository == name and (r.tag == arg or d == arg):
                        md = d
                        break
            if md is None:
                return _err(404, "MANIFEST_UNKNOWN", f"manifest unknown: {name}:{arg}")
            body = self.store.read_blob(md)
            mt = json.loads(body).get("mediaType") or "application/vnd.oci.image.manifest.v1+json"
            return Response(200, b"" if req.method == "HEAD" else body, mt, {"Docker-Content-Digest": md})
        try:
            body = self.store.read_blob(arg)
        except (OSError, ValueError):
            return _err(404, "BLOB_UNKNOWN", f"blob unknown: {arg}")
        return Response(200, b"" if req.method == "HEAD" else body, "application/octet-stream",
                        {"Docker-Content-Digest": arg})
