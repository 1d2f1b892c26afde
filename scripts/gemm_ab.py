"""A/B the bf16 GEMM kernels (random uniform operands, fp32 out) on cuda:0."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubernetes_amd.ops import hip_kernels as h  # noqa: E402

for size, iters in ((4096, 30), (8192, 10)):
    for path in (1, 2, 0, 2, 0):
        h.set_gemm_path(path)
        r = h.diag_mfma(0, size, iters)
        name = {0: "256-8phase", 1: "128-regstage", 2: "256-glds-2barrier"}[path]
        print(f"{size}^3 path={name}: {r['tflops']:.1f} TF/s, max_rel_err={r['max_rel_err']:.2e}", flush=True)
h.set_gemm_path(0)
