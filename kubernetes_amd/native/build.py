"""Build every native component in-tree (C++ with g++, HIP for gfx950 with hipcc).

    python -m kubernetes_amd.native.build [--force] [--only NAME]

Targets land in kubernetes_amd/native/{lib,bin}/ so they travel with the repo snapshot to
the GPU box (git-ignored, not gpurun-ignored). Incremental: a target is rebuilt only when a
source is newer than it.
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

from . import BIN_DIR, LIB_DIR, SRC_DIR

ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")
ARCH = os.environ.get("KAMD_OFFLOAD_ARCH", "gfx950")


def _s(*p):
    return os.path.join(SRC_DIR, *p)


def _py_ext():
    import sysconfig
    return sysconfig.get_paths()["include"], sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def targets():
    cxx = ["g++", "-O2", "-std=c++17", "-Wall", "-fPIC"]
    py_inc, ext = _py_ext()
    hip = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC"]
    return {
        "kamd_smi": ([_s("amdsmi_shim", "kamd_smi.cc"), _s("amdsmi_shim", "kamd_smi.h")],
                     os.path.join(LIB_DIR, "libkamd_smi.so"),
                     cxx + ["-shared", f"-I{ROCM}/include", _s("amdsmi_shim", "kamd_smi.cc"), "-ldl"]),
        "kamd_store": ([_s("store", "mvcc_store.cc")], os.path.join(LIB_DIR, "libkamd_store.so"),
                       cxx + ["-O3", "-shared", _s("store", "mvcc_store.cc")]),
        "kamd_etcd": ([_s("store", "mvcc_store.cc"), _s("pbcodec", "pb_codec.h")], os.path.join(BIN_DIR, "kamd-etcd"),
                      cxx + ["-O3", "-pthread", "-DKAMD_STORE_SERVER", _s("store", "mvcc_store.cc")]),
        # the API server's protobuf storage codec (CPython extension over native/pbcodec/pb_codec.h)
        "kamd_pbcodec": ([_s("pbcodec", "kamd_pbcodec.cc"), _s("pbcodec", "pb_codec.h")],
                         os.path.join(LIB_DIR, "_kamd_pbcodec" + ext),
                         cxx + ["-O3", "-shared", f"-I{py_inc}", _s("pbcodec", "kamd_pbcodec.cc")]),
        "kamd_oci": ([_s("oci", "oci_devices.cc")], os.path.join(LIB_DIR, "libkamd_oci.so"),
                     cxx + ["-shared", _s("oci", "oci_devices.cc")]),
        "kamd_crypto": ([_s("crypto", "kamd_crypto.cc")], os.path.join(LIB_DIR, "libkamd_crypto.so"),
                        cxx + ["-O2", "-shared", _s("crypto", "kamd_crypto.cc"), "-lcrypto"]),
        "pause": ([_s("pause", "pause.cc")], os.path.join(BIN_DIR, "pause"),
                  ["g++", "-Os", "-Wall", "-Werror", "-static", _s("pause", "pause.cc")]),
        "container_init": ([_s("pause", "container_init.cc")], os.path.join(BIN_DIR, "container-init"),
                           ["g++", "-O2", "-Wall", "-Werror", "-static", _s("pause", "container_init.cc")]),
        "kamd_runc": ([_s("runc", "kamd_runc.cc")], os.path.join(BIN_DIR, "kamd-runc"),
                      ["g++", "-O2", "-std=c++17", "-Wall", "-Werror", "-static", _s("runc", "kamd_runc.cc")]),
        # preloaded by kamd-runc into Landlock-tier containers (EACCES -> EPERM on /dev/dri)
        "kamd_devshim": ([_s("runc", "kamd_devshim.cc")], os.path.join(LIB_DIR, "libkamd_devshim.so"),
                         cxx + ["-shared", "-Wextra", "-Werror", _s("runc", "kamd_devshim.cc"), "-ldl"]),
        "orphan": ([_s("pause", "orphan.cc")], os.path.join(BIN_DIR, "orphan"),
                   ["g++", "-Os", "-Wall", _s("pause", "orphan.cc")]),
        "kamd_hip": ([_s("hip", "kamd_hip.hip")], os.path.join(LIB_DIR, "libkamd_hip.so"),
                     hip + ["-shared", _s("hip", "kamd_hip.hip")]),
        "hip_vector_add": ([_s("hip", "vector_add_main.hip"), _s("hip", "kamd_hip.hip")],
                           os.path.join(BIN_DIR, "hip-vector-add"),
                           hip + [_s("hip", "vector_add_main.hip"), _s("hip", "kamd_hip.hip")]),
        "xgmi_probe": ([_s("hip", "xgmi_probe.cc")], os.path.join(BIN_DIR, "xgmi-probe"),
                       [HIPCC, f"--offload-arch={ARCH}", "-O2", "-x", "hip", _s("hip", "xgmi_probe.cc"),
                        f"-I{ROCM}/include", f"-L{ROCM}/lib", "-lrccl", f"-Wl,-rpath,{ROCM}/lib"]),
    }


SAN_DIR = os.path.join(os.path.dirname(BIN_DIR), "san")
SAN_FLAGS = {
    # host-code sanitizers only: GPU-side ASan / xnack+ code objects are not available on the MI355X pool
    "asan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer"],
    "tsan": ["-fsanitize=thread"],
}


def sanitizer_targets():
    """Sanitized builds of the native host code (SURVEY §5.2 race detection: the reference's
    `KUBE_RACE=-race`): ASan+UBSan for the store engine/server, TSan for the multi-threaded
    AMD SMI shim. Output under kubernetes_amd/native/san/<kind>/."""
    base = ["g++", "-O1", "-g", "-std=c++17", "-Wall"]
    asan, tsan = os.path.join(SAN_DIR, "asan"), os.path.join(SAN_DIR, "tsan")
    store = _s("store", "mvcc_store.cc")
    return {
        "asan_kamd_etcd": ([store, _s("pbcodec", "pb_codec.h")], os.path.join(asan, "kamd-etcd"),
                           base + SAN_FLAGS["asan"] + ["-pthread", "-DKAMD_STORE_SERVER", store]),
        # the store thread and the watch fan-out thread share the event queue and KV lifetimes
        "tsan_kamd_etcd": ([store, _s("pbcodec", "pb_codec.h")], os.path.join(tsan, "kamd-etcd"),
                           base + SAN_FLAGS["tsan"] + ["-pthread", "-DKAMD_STORE_SERVER", store]),
        "asan_store_fuzz": ([store, _s("tests", "store_fuzz.cc")], os.path.join(asan, "store_fuzz"),
                            base + SAN_FLAGS["asan"] + [_s("tests", "store_fuzz.cc")]),
        "tsan_smi_threads": ([_s("amdsmi_shim", "kamd_smi.cc"), _s("amdsmi_shim", "kamd_smi.h"), _s("tests", "smi_threads.cc")],
                             os.path.join(tsan, "smi_threads"),
                             base + SAN_FLAGS["tsan"] + [f"-I{ROCM}/include", _s("tests", "smi_threads.cc"),
                                                         _s("amdsmi_shim", "kamd_smi.cc"), "-ldl", "-lpthread"]),
    }


def _stale(srcs, out):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.exists(s) and os.path.getmtime(s) > t for s in srcs)


def build(force=False, only=None, verbose=True, sanitize=False):
    os.makedirs(LIB_DIR, exist_ok=True)
    os.makedirs(BIN_DIR, exist_ok=True)
    jobs = []
    tg = sanitizer_targets() if sanitize else targets()
    for name, (srcs, out, cmd) in tg.items():
        os.makedirs(os.path.dirname(out), exist_ok=True)
        if only and name not in only:
            continue
        if not all(os.path.exists(s) for s in srcs if s.endswith((".cc", ".hip"))):
            continue
        if force or _stale(srcs, out):
            jobs.append((name, out, cmd + ["-o", out]))
    failures = []

    def run(job):
        name, out, cmd = job
        r = subprocess.run(cmd, capture_output=True, text=True)
        return name, out, r

    with ThreadPoolExecutor(max_workers=min(8, max(1, len(jobs)))) as ex:
        for name, out, r in ex.map(run, jobs):
            if r.returncode != 0:
                failures.append(name)
                print(f"[build] {name} FAILED\n{r.stderr[-4000:]}", file=sys.stderr)
            elif verbose:
                print(f"[build] {name} -> {os.path.relpath(out)}")
    if failures:
        raise RuntimeError(f"native build failed: {failures}")
    return [j[1] for j in jobs]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only", nargs="*")
    ap.add_argument("--sanitize", action="store_true", help="build the ASan/UBSan/TSan variants + native test drivers")
    a = ap.parse_args()
    build(a.force, a.only, sanitize=a.sanitize)


if __name__ == "__main__":
    main()
