"""Locate wrong output regions of the 8-phase GEMM by wave / quadrant (debug aid)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubernetes_amd.ops import hip_kernels as h  # noqa: E402

h.set_gemm_path(0)
for M, N, K in ((256, 256, 128), (256, 256, 192), (256, 256, 256), (256, 256, 512), (512, 512, 1024), (4096, 4096, 4096)):
    torch.manual_seed(0)
    a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    ref = a.float() @ b.float().T
    out = h.gemm_bf16_nt(a, b, out_fp32=True)
    bad = ((out - ref).abs() > 2e-3 * K ** 0.5 + 2e-3 * ref.abs())
    r = torch.arange(M, device="cuda")[:, None].expand(M, N)
    c = torch.arange(N, device="cuda")[None, :].expand(M, N)
    key = ((r % 256) // 128) * 1000 + ((r % 128) // 64) * 100 + ((c % 256) // 64) * 10 + ((c % 64) // 32)
    ks = sorted(set(key[bad].tolist()))
    print(f"{M}x{N}x{K}: bad={bad.float().mean().item():.3f} regions(wr,mq,wc,nq)={ks[:40]}", flush=True)
