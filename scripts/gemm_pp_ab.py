"""Ping-pong GEMM (path 3) vs the 8-phase kernel (path 0) vs torch.matmul: correctness against an
fp32 torch reference on several shapes, then throughput (uniform random operands, fp32 out)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from kubernetes_amd.ops import hip_kernels as h  # noqa: E402

torch.manual_seed(0)
dev = "cuda:0"
for (m, n, k) in ((256, 256, 64), (512, 768, 128), (1024, 512, 320), (2048, 2048, 2048)):
    a = (torch.rand(m, k, device=dev) * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(n, k, device=dev) * 2 - 1).to(torch.bfloat16)
    ref = a.float() @ b.float().t()
    for path in (6, 5, 4, 3, 7):
        h.set_gemm_path(path)
        c = h.gemm_bf16_nt(a, b)
        torch.cuda.synchronize()
        err = ((c - ref).abs().max() / ref.abs().max()).item()
        cb = h.gemm_bf16_nt(a, b, out_fp32=False).float()
        torch.cuda.synchronize()
        errb = ((cb - ref).abs().max() / ref.abs().max()).item()
        print(f"check {m}x{n}x{k} path={path}: max_rel_err={err:.2e} (bf16 out {errb:.2e})", flush=True)
        assert err < 1e-2 and errb < 2e-2, (m, n, k, path, err, errb)


def bench(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


for size, iters in ((4096, 50), (8192, 20), (16384, 5)):
    kdim = 8192 if size == 16384 else size
    a = (torch.rand(size, kdim, device=dev) * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(size, kdim, device=dev) * 2 - 1).to(torch.bfloat16)
    flops = 2.0 * size * size * kdim
    out = {}
    for rep in range(2):
        for path in (6, 5, 4, 3, 7):
            h.set_gemm_path(path)
            dt = bench(lambda: h.gemm_bf16_nt(a, b), iters)
            out.setdefault(path, []).append(flops / dt / 1e12)
        dt = bench(lambda: a @ b.t(), iters)
        out.setdefault("torch", []).append(flops / dt / 1e12)
    best = max(max(out[p]) for p in (3, 4, 5, 6))
    print(f"{size}x{size}x{kdim}: pp {max(out[3]):.0f}  pp+epi {max(out[4]):.0f}  pp+prio {max(out[5]):.0f}  "
          f"pp+both {max(out[6]):.0f}  8-phase {max(out[7]):.0f}  torch {max(out['torch']):.0f} TF/s  "
          f"best/torch {best / max(out['torch']):.2f}", flush=True)
h.set_gemm_path(0)
