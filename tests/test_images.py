"""Container images: references, the OCI store (layers, whiteouts, rootfs confinement), Registry
v2 pulls with bearer-token auth and pull-secret keyrings, and pods running an image's entrypoint
on an overlay of its unpacked layers.

Parity: `pkg/kubelet/images/image_manager_test.go` (pull policy / back-off, covered with the
kubelet tests), `pkg/credentialprovider/keyring_test.go` (URL matching), `pkg/util/parsers`
(ParseImageName), and the e2e "should be able to pull image from docker hub / private registry
with secret" (`test/e2e/common/runtime.go`) — here against a local registry server, the only
registry reachable without network.
"""
import base64
import gzip
import io
import json
import os
import subprocess
import tarfile

import pytest

from kubernetes_amd.cluster import LocalCluster
from kubernetes_amd.images import reference
from kubernetes_amd.images.credentials import keyring_from_secrets
from kubernetes_amd.images.registry import Auth, RegistryClient, RegistryError
from kubernetes_amd.images.registry_server import RegistryServer
from kubernetes_amd.images.service import ImageService, command_for, node_image_service
from kubernetes_amd.images.store import OCIStore, apply_layer, build_image, sha256_digest
from kubernetes_amd.kubelet.runtime.process import runc_features


def test_reference_parsing():
    cases = {
        "busybox": ("docker.io", "library/busybox", "latest", None),
        "amd/rocm:6.2": ("docker.io", "amd/rocm", "6.2", None),
        "localhost:5000/a/b": ("localhost:5000", "a/b", "latest", None),
        "registry.local/x@sha256:" + "ab" * 32: ("registry.local", "x", None, "sha256:" + "ab" * 32),
        "index.docker.io/library/busybox:1.28": ("docker.io", "library/busybox", "1.28", None),
    }
    for s, want in cases.items():
        r = reference.parse(s)
        assert (r.registry, r.repository, r.tag, r.digest) == want, s
    assert reference.parse("busybox").familiar() == "busybox:latest"
    for bad in ("Busybox", "a//b", "x:bad tag", ""):
        with pytest.raises(reference.InvalidReference):
            reference.parse(bad)


def _layer(entries):
    """entries: (name, kind, payload) with kind file|dir|symlink|hardlink."""
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w") as tf:
        for name, kind, payload in entries:
            ti = tarfile.TarInfo(name)
            if kind == "dir":
                ti.type, ti.mode = tarfile.DIRTYPE, 0o755
                tf.addfile(ti)
            elif kind == "symlink":
                ti.type, ti.linkname = tarfile.SYMTYPE, payload
                tf.addfile(ti)
            elif kind == "hardlink":
                ti.type, ti.linkname = tarfile.LNKTYPE, payload
                tf.addfile(ti)
            else:
                ti.size, ti.mode = len(payload), 0o644
                tf.addfile(ti, io.BytesIO(payload))
    return gzip.compress(buf.getvalue())


def test_layers_whiteouts_and_confinement(tmp_path):
    root = tmp_path / "rootfs"
    root.mkdir()
    outside = tmp_path / "outside"
    outside.mkdir()
    apply_layer(str(root), io.BytesIO(_layer([
        ("etc", "dir", None), ("etc/keep", "file", b"1"), ("etc/drop", "file", b"2"),
        ("opt/a/x", "file", b"x"), ("opt/a/y", "file", b"y"), ("./.profile", "file", b"dot"),
        ("escape", "symlink", str(outside)),          # an absolute link pointing out of the root
        ("up", "symlink", "../../.."),
    ])))
    apply_layer(str(root), io.BytesIO(_layer([
        ("etc/.wh.drop", "file", b""),                # whiteout
        ("opt/a/.wh..wh..opq", "file", b""),          # opaque directory
        ("opt/a/z", "file", b"z"),
        ("escape/pwned", "file", b"no"),              # must land inside the root
        ("up/etc/pwned2", "file", b"no"),
        ("etc/link", "hardlink", "etc/keep"),
    ])))
    assert sorted(os.listdir(root / "etc")) == ["keep", "link", "pwned2"]     # "up" resolved to the root
    assert sorted(os.listdir(root / "opt" / "a")) == ["z"]
    assert (root / ".profile").read_bytes() == b"dot"
    assert os.listdir(outside) == []
    assert (root / str(outside).lstrip("/") / "pwned").read_bytes() == b"no"
    assert (root / "etc" / "pwned2").read_bytes() == b"no"
    assert os.stat(root / "etc" / "link").st_ino == os.stat(root / "etc" / "keep").st_ino


@pytest.mark.parametrize("entry", [".wh..", ".wh...", "..", "a/..", "a/.wh..", "a/.wh...", "./..", "a/b/../.."])
def test_dot_entries_cannot_touch_the_store(tmp_path, entry):
    """A hostile layer naming '.', '..' or a whiteout of them must not remove or write the
    directory above the layer root (the store's other unpacked images)."""
    store = tmp_path / "rootfs"
    root = store / "img1"
    sibling = store / "img2"
    root.mkdir(parents=True)
    sibling.mkdir()
    (sibling / "bin").write_bytes(b"other image")
    (root / "a").mkdir()
    (root / "a" / "f").write_bytes(b"keep")
    with pytest.raises(ValueError):
        apply_layer(str(root), io.BytesIO(_layer([(entry, "file", b"x")])))
    assert (sibling / "bin").read_bytes() == b"other image"
    assert (root / "a" / "f").read_bytes() == b"keep"
    assert sorted(os.listdir(store)) == ["img1", "img2"]


def test_store_tags_gc_and_layout_import(tmp_path):
    st = OCIStore(str(tmp_path / "s"))
    md = build_image(st, "registry.local/base:1", {"bin/tool": (b"#!x", 0o755)}, {"Entrypoint": ["/bin/tool"]})
    md2 = build_image(st, "registry.local/app:2", {"app.txt": b"hello"}, {"Cmd": ["run"], "Env": ["A=1"]},
                      base="registry.local/base:1")
    img = st.image("registry.local/app:2")
    assert img["repo_tags"] == ["registry.local/app:2"] and img["manifest_digest"] == md2
    assert img["config"]["config"] == {"Entrypoint": ["/bin/tool"], "Cmd": ["run"], "Env": ["A=1"]}
    rf = st.rootfs("registry.local/app:2")
    assert open(os.path.join(rf, "app.txt")).read() == "hello" and os.access(os.path.join(rf, "bin/tool"), os.X_OK)
    assert st.resolve(f"registry.local/app@{md2}") == md2 and st.resolve(img["id"]) == md2
    # removing the base keeps the shared layer (app still uses it)
    base_layer = st.manifest(md)["layers"][0]["digest"]
    st.remove("registry.local/base:1")
    assert st.has_blob(base_layer) and st.image("registry.local/base:1") is None
    st.remove("registry.local/app:2")
    assert not st.has_blob(base_layer) and not os.listdir(st.rootfs_dir)
    # OCI image layout export -> import (air-gapped node)
    src = OCIStore(str(tmp_path / "src"))
    m = build_image(src, "registry.local/x:1", {"f": b"1"})
    lay = tmp_path / "layout"
    (lay / "blobs" / "sha256").mkdir(parents=True)
    for h in os.listdir(src.blob_dir):
        (lay / "blobs" / "sha256" / h).write_bytes(open(os.path.join(src.blob_dir, h), "rb").read())
    (lay / "oci-layout").write_text('{"imageLayoutVersion": "1.0.0"}')
    (lay / "index.json").write_text(json.dumps({"schemaVersion": 2, "manifests": [
        {"mediaType": "application/vnd.oci.image.manifest.v1+json", "digest": m, "size": 1,
         "annotations": {"org.opencontainers.image.ref.name": "registry.local/x:1"}}]}))
    dst = OCIStore(str(tmp_path / "dst"))
    assert dst.import_layout(str(lay)) == ["registry.local/x:1"]
    assert dst.image("registry.local/x:1")["manifest_digest"] == m


def test_command_resolution_table():
    """The Kubernetes command/args vs ENTRYPOINT/CMD table (`tasks/inject-data-application`)."""
    cfg = {"Entrypoint": ["/ep"], "Cmd": ["c1"]}
    assert command_for({}, cfg) == ["/ep", "c1"]
    assert command_for({"command": ["/x"]}, cfg) == ["/x"]
    assert command_for({"args": ["a"]}, cfg) == ["/ep", "a"]
    assert command_for({"command": ["/x"], "args": ["a"]}, cfg) == ["/x", "a"]


def test_keyring_matching():
    def secret(kind, auths):
        if kind == "json":
            return {"type": "kubernetes.io/dockerconfigjson", "data": {".dockerconfigjson": base64.b64encode(
                json.dumps({"auths": auths}).encode()).decode()}}
        return {"type": "kubernetes.io/dockercfg", "data": {".dockercfg": base64.b64encode(json.dumps(auths).encode()).decode()}}
    kr = keyring_from_secrets([
        secret("json", {"https://index.docker.io/v1/": {"username": "hub", "password": "p"},
                        "registry.local:5000": {"auth": base64.b64encode(b"loc:pw").decode()},
                        "*.corp.example": {"username": "wild", "password": "w"}}),
        secret("cfg", {"registry.local:5000/team": {"username": "team", "password": "t"}}),
    ])
    assert [a.username for a in kr.lookup("busybox")] == ["hub"]
    assert [a.username for a in kr.lookup("registry.local:5000/team/app")] == ["team", "loc"]
    assert [(a.username, a.password) for a in kr.lookup("registry.local:5000/other")] == [("loc", "pw")]
    assert [a.username for a in kr.lookup("img.corp.example/x")] == ["wild"]
    assert kr.lookup("registry.local/x") == [] and kr.lookup("a.b.corp.example/x") == []


def test_registry_pull_with_token_auth_index_and_digest(run, tmp_path):
    async def main():
        served = OCIStore(str(tmp_path / "served"))
        md = build_image(served, "127.0.0.1/ml/train:v1", {"w.bin": os.urandom(200000)}, {"Cmd": ["go"]})
        # a multi-platform index naming the amd64 manifest
        man = served.read_blob(md)
        index = json.dumps({"schemaVersion": 2, "mediaType": "application/vnd.oci.image.index.v1+json", "manifests": [
            {"mediaType": "application/vnd.oci.image.manifest.v1+json", "digest": sha256_digest(b"nope"), "size": 4,
             "platform": {"os": "linux", "architecture": "s390x"}},
            {"mediaType": "application/vnd.oci.image.manifest.v1+json", "digest": md, "size": len(man),
             "platform": {"os": "linux", "architecture": "amd64"}}]}).encode()
        idx = served.put_blob(index)
        served.tag("127.0.0.1/ml/train:multi", idx)
        srv = await RegistryServer(served, users={"alice": "s3cret"}).start()
        try:
            host = srv.address
            cli = RegistryClient()
            dst = OCIStore(str(tmp_path / "node"))
            with pytest.raises(RegistryError) as ei:
                await cli.pull(f"{host}/ml/train:v1", dst)
            assert ei.value.status == 401
            with pytest.raises(RegistryError):
                await cli.pull(f"{host}/ml/train:v1", dst, Auth("alice", "wrong"))
            got = await cli.pull(f"{host}/ml/train:v1", dst, Auth("alice", "s3cret"))
            assert got == md and dst.image(f"{host}/ml/train:v1")["config"]["config"] == {"Cmd": ["go"]}
            assert await cli.pull(f"{host}/ml/train:multi", dst, Auth("alice", "s3cret")) == md
            pinned = f"{host}/ml/train@{idx}"
            assert await cli.pull(pinned, dst, Auth("alice", "s3cret")) == md
            assert dst.image(pinned)["manifest_digest"] == md
            with pytest.raises(RegistryError) as ei:
                await cli.pull(f"{host}/ml/missing:v1", dst, Auth("alice", "s3cret"))
            assert ei.value.status == 404
        finally:
            await srv.stop()
    run(main())


def _static_tool(path):
    """A static binary (the image's only content) printing a file, its uid and cwd."""
    src = path.with_suffix(".c")
    src.write_text('#include <stdio.h>\n#include <stdlib.h>\n#include <unistd.h>\n'
                   'int main(int c,char**v){char b[256],w[256];FILE*f=fopen(v[1],"r");if(!f){puts("nofile");return 3;}'
                   'size_t n=fread(b,1,255,f);b[n]=0;printf("%s|uid=%d|cwd=%s|A=%s\\n",b,getuid(),getcwd(w,256),'
                   'getenv("A")?getenv("A"):"");return 0;}\n')
    subprocess.run(["gcc", "-static", "-O1", "-o", str(path), str(src)], check=True)
    return path.read_bytes()


@pytest.mark.skipif(not runc_features().get("isolation"), reason="needs mount namespaces (root)")
def test_pod_runs_image_entrypoint_on_overlay_rootfs_with_pull_secret(run, tmp_path):
    async def main():
        served = OCIStore(str(tmp_path / "served"))
        tool = _static_tool(tmp_path / "show")
        build_image(served, "127.0.0.1/tools/show:v1", {"bin/show": (tool, 0o755), "data/msg": b"from-the-image",
                                                        "etc/passwd": b"root:x:0:0::/:\nsvc:x:1234:1234::/:\n"},
                    {"Entrypoint": ["/bin/show"], "Cmd": ["/data/msg"], "Env": ["A=image", "PATH=/bin"],
                     "WorkingDir": "/data", "User": "svc"})
        srv = await RegistryServer(served, users={"bob": "pw"}).start()
        cl = LocalCluster(nodes=1, gpus_per_node=0, runtime="process", workdir=str(tmp_path / "c"),
                          kubelet_http=True, image_service=lambda d: node_image_service(d))
        await cl.start()
        try:
            c = cl.client
            await c.create("secrets", {"metadata": {"name": "regcred", "namespace": "default"},
                                       "type": "kubernetes.io/dockerconfigjson",
                                       "data": {".dockerconfigjson": base64.b64encode(json.dumps({"auths": {
                                           srv.address: {"username": "bob", "password": "pw"}}}).encode()).decode()}})
            img = f"{srv.address}/tools/show:v1"
            for name, extra in (("img", {}), ("img-args", {"args": ["/etc/passwd"], "env": [{"name": "A", "value": "pod"}]})):
                await c.create("pods", {"metadata": {"name": name, "namespace": "default"}, "spec": {
                    "restartPolicy": "Never", "imagePullSecrets": [{"name": "regcred"}],
                    "containers": [dict({"name": "c", "image": img, "imagePullPolicy": "Always"}, **extra)]}})

            async def done(name):
                p = await c.get("pods", name, "default")
                return p if p["status"].get("phase") in ("Succeeded", "Failed") else None
            p = await cl.wait_for(lambda: done("img"), timeout=30)
            assert p["status"]["phase"] == "Succeeded", p["status"]["containerStatuses"]
            st, logs = await c.http.request("GET", "/api/v1/namespaces/default/pods/img/log")
            assert logs.decode().strip() == "from-the-image|uid=1234|cwd=/data|A=image"
            await cl.wait_for(lambda: done("img-args"), timeout=30)
            st, logs = await c.http.request("GET", "/api/v1/namespaces/default/pods/img-args/log")
            assert logs.decode().startswith("root:x:0:0::/:\nsvc:x:1234:1234::/:\n|uid=1234|cwd=/data|A=pod")
            events = (await c.list("events", "default"))["items"]
            assert any(e["reason"] == "Pulled" and "Successfully pulled" in e["message"] for e in events)
            # no credentials and pull policy Always -> ErrImagePull (IfNotPresent would use the cached image)
            await c.create("pods", {"metadata": {"name": "nocred", "namespace": "default"}, "spec": {
                "containers": [{"name": "c", "image": img, "imagePullPolicy": "Always"}]}})

            async def pull_err():
                p = await c.get("pods", "nocred", "default")
                w = ((p["status"].get("containerStatuses") or [{}])[0].get("state") or {}).get("waiting") or {}
                return w.get("reason") in ("ErrImagePull", "ImagePullBackOff")
            await cl.wait_for(pull_err, timeout=30)
        finally:
            await cl.stop()
            await srv.stop()
    run(main(), timeout=90)


def test_kamd_image_cli(tmp_path):
    from kubernetes_amd.cmd.image import main
    src = OCIStore(str(tmp_path / "src"))
    m = build_image(src, "registry.local/cli:1", {"f": b"1"})
    lay = tmp_path / "layout.tar"
    with tarfile.open(lay, "w") as tf:
        def add(name, data):
            ti = tarfile.TarInfo(name)
            ti.size = len(data)
            tf.addfile(ti, io.BytesIO(data))
        add("oci-layout", b'{"imageLayoutVersion": "1.0.0"}')
        add("index.json", json.dumps({"schemaVersion": 2, "manifests": [
            {"mediaType": "application/vnd.oci.image.manifest.v1+json", "digest": m, "size": 1}]}).encode())
        for h in os.listdir(src.blob_dir):
            add("blobs/sha256/" + h, open(os.path.join(src.blob_dir, h), "rb").read())
    root = str(tmp_path / "node")
    out = io.StringIO()
    assert main(["--root", root, "import", str(lay), "--tag", "registry.local/cli:1"], out) == 0
    assert main(["--root", root, "ls"], out) == 0
    assert "registry.local/cli:1" in out.getvalue()
    assert main(["--root", root, "rm", "registry.local/cli:1"], out) == 0
    assert OCIStore(root).images() == []
