"""kamd-image: manage a node's OCI image store and run the in-cluster registry add-on.

    python -m kubernetes_amd.cmd.image --root /var/lib/kubelet/images ls
    python -m kubernetes_amd.cmd.image --root ... pull registry.local:5000/ml/train:v1 [--insecure-registry H]
    python -m kubernetes_amd.cmd.image --root ... import image-layout.tar [--tag name:tag]
    python -m kubernetes_amd.cmd.image --root ... rm busybox:1.28
    python -m kubernetes_amd.cmd.image --root ... serve --address 0.0.0.0 --port 5000

The store is the one the kubelet / kamd-cri use (`--image-service oci`): images imported here are
present for `imagePullPolicy: IfNotPresent` pods without any registry (air-gapped nodes), and
`serve` exposes a store read-only over the Registry v2 API (the role of the reference's
`cluster/addons/registry`).
"""
from __future__ import annotations

import argparse
import asyncio
import os
import sys

from ..images.registry import Auth, RegistryClient
from ..images.registry_server import RegistryServer
from ..images.store import OCIStore
from ._common import run_until_signal, setup_logging


def main(argv=None, out=sys.stdout):
    ap = argparse.ArgumentParser("kamd-image")
    ap.add_argument("--root", default="/var/lib/kubelet/images")
    ap.add_argument("-v", type=int, default=0)
    sub = ap.add_subparsers(dest="cmd", required=True)
    sub.add_parser("ls")
    p = sub.add_parser("pull")
    p.add_argument("image")
    p.add_argument("--insecure-registry", action="append", default=[])
    p.add_argument("--username", default="")
    p.add_argument("--password", default=os.environ.get("KAMD_REGISTRY_PASSWORD", ""))
    i = sub.add_parser("import")
    i.add_argument("path", help="OCI image layout (directory or tar)")
    i.add_argument("--tag", default=None)
    r = sub.add_parser("rm")
    r.add_argument("image")
    s = sub.add_parser("serve")
    s.add_argument("--address", default="127.0.0.1")
    s.add_argument("--port", type=int, default=5000)
    a = ap.parse_args(argv)
    setup_logging(a.v)
    store = OCIStore(a.root)
    if a.cmd == "ls":
        print(f"{'IMAGE':60} {'ID':20} SIZE", file=out)
        for img in store.images():
            for t in img["repo_tags"] or ["<none>"]:
                print(f"{t:60} {img['id'][7:19]:20} {img['size']}", file=out)
        return 0
    if a.cmd == "pull":
        auth = Auth(a.username, a.password) if a.username else None
        md = asyncio.run(RegistryClient(a.insecure_registry).pull(a.image, store, auth))
        print(f"{a.image}: {md}", file=out)
        return 0
    if a.cmd == "import":
        for t in store.import_layout(a.path, a.tag):
            print(f"imported {t}", file=out)
        return 0
    if a.cmd == "rm":
        if not store.remove(a.image):
            print(f"error: no such image: {a.image}", file=sys.stderr)
            return 1
        print(f"untagged {a.image}", file=out)
        return 0

    async def start():
        srv = await RegistryServer(store, a.address).start(a.port)
        print(f"kamd-image registry serving {a.root} on http://{srv.address}/v2/", flush=True)
        return srv
    run_until_signal(start)
    return 0


if __name__ == "__main__":
    sys.exit(main())
