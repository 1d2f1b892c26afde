"""kamd-cri: a standalone CRI (v1alpha1) runtime daemon on a unix socket — the role the
dockershim's gRPC endpoint plays for the reference kubelet (`unix:///var/run/dockershim.sock`,
`cmd/kubelet/app/options/options.go:196`; `pkg/kubelet/dockershim/remote/docker_server.go`).

    python -m kubernetes_amd.cmd.cri --listen /var/run/kamd-cri.sock --runtime process
    python -m kubernetes_amd.cmd.kubelet --container-runtime remote \
        --container-runtime-endpoint unix:///var/run/kamd-cri.sock ...
"""
from __future__ import annotations

import argparse
import os

from ..cri.server import CRIServer
from ..kubelet.runtime.process import ProcessRuntime
from ..kubelet.runtime.stub import StubRuntime
from ._common import run_until_signal, setup_logging


def main(argv=None):
    ap = argparse.ArgumentParser("kamd-cri")
    ap.add_argument("--listen", default="/var/run/kamd-cri.sock")
    ap.add_argument("--runtime", default="process", choices=["process", "stub"])
    ap.add_argument("--root-dir", default="/var/lib/kamd-cri")
    ap.add_argument("--hooks-dir", default=None,
                    help="runtime hooks (JSON {runtime, annotations, images}) choosing a runtime per container "
                         "(the fork's dockershim hooks.d); both runtimes are then available")
    ap.add_argument("--image-service", default="oci", choices=["oci", "builtin"],
                    help="'oci' = OCI store + registry pulls, 'builtin' = built-in images / host root only")
    ap.add_argument("--insecure-registry", action="append", default=[])
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    setup_logging(a.v)

    async def start():
        images = None
        if a.image_service == "oci" and a.runtime == "process":
            from ..images.service import node_image_service
            images = node_image_service(os.path.join(a.root_dir, "images"), True, a.insecure_registry)
        rt = ProcessRuntime(os.path.join(a.root_dir, "containers"), images=images) if a.runtime == "process" \
            else StubRuntime()
        hook_task = None
        if a.hooks_dir:
            import asyncio

            from ..kubelet.runtime.hooks import HookedRuntime, HookService
            runtimes = {"process": rt if a.runtime == "process" else ProcessRuntime(os.path.join(a.root_dir, "containers")),
                        "stub": rt if a.runtime == "stub" else StubRuntime()}
            hooks = HookService(a.hooks_dir, available_runtimes=runtimes).load()
            rt = HookedRuntime(runtimes, a.runtime, hooks)
            hook_task = asyncio.ensure_future(hooks.watch())
        os.makedirs(os.path.dirname(os.path.abspath(a.listen)), exist_ok=True)
        srv = await CRIServer(rt, a.listen, checkpoint_dir=os.path.join(a.root_dir, "sandbox")).start()
        srv.hook_task = hook_task
        print(f"kamd-cri serving CRI v1alpha1 ({rt.name} runtime) on unix://{a.listen}, "
              f"streaming on 127.0.0.1:{srv.streaming.port}", flush=True)
        return srv

    run_until_signal(start)


if __name__ == "__main__":
    main()
