"""Our MFMA GEMM vs torch.matmul (hipBLASLt) on cuda:0, bf16 in, bf16 out, C = A @ B^T."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubernetes_amd.ops import hip_kernels as h  # noqa: E402


def bench(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


for m, n, k in ((4096, 4096, 4096), (8192, 8192, 8192), (16384, 16384, 8192)):
    a = (torch.rand(m, k, device="cuda") * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(n, k, device="cuda") * 2 - 1).to(torch.bfloat16)
    iters = 20 if m <= 8192 else 5
    flop = 2.0 * m * n * k
    t_torch = bench(lambda: torch.matmul(a, b.T), iters)
    t_ours = bench(lambda: h.gemm_bf16_nt(a, b, out_fp32=False), iters)
    ref = torch.matmul(a.float(), b.float().T)
    err = ((h.gemm_bf16_nt(a, b, out_fp32=False).float() - ref).abs().max() / ref.abs().max()).item()
    print(f"{m}x{n}x{k}: torch {flop / t_torch / 1e9:.0f} TF/s ({t_torch:.3f} ms)  ours {flop / t_ours / 1e9:.0f} TF/s "
          f"({t_ours:.3f} ms)  ratio {t_torch / t_ours:.2f}  max_rel_err {err:.1e}", flush=True)
