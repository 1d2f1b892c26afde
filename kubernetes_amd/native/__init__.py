"""Native (C++ / HIP) components and their Python bindings.

Built in-tree by `python -m kubernetes_amd.native.build` (also `__graft_entry__.build()`):
  lib/libkamd_smi.so     AMD SMI shim (native/amdsmi_shim)
  lib/libkamd_store.so   MVCC KV engine (native/store)
  lib/libkamd_oci.so     OCI device-injection helper (native/oci)
  lib/libkamd_crypto.so  AES-CBC/GCM, NaCl secretbox, x509 issue/verify (native/crypto, OpenSSL)
  lib/libkamd_hip.so     HIP/CDNA4 kernels: vector_add, MFMA diag GEMM, HBM bandwidth (gfx950)
  bin/pause, bin/orphan  pod-sandbox PID 1 and its reaper test helper (native/pause)
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(HERE, "lib")
BIN_DIR = os.path.join(HERE, "bin")
REPO = os.path.dirname(os.path.dirname(HERE))
SRC_DIR = os.path.join(REPO, "native")
