"""HIP kernels on a real MI355X, checked against plain PyTorch fp32 references."""
import os

import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hk():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from kubernetes_amd.ops import hip_kernels
    hip_kernels.load()  # must load: no fallback
    return hip_kernels


def test_device_is_gfx950(hk):
    assert hk.device_arch(0).startswith("gfx950")


def test_vector_add_matches_torch(hk):
    a = torch.randn(50000, device="cuda")
    b = torch.randn(50000, device="cuda")
    c = hk.vector_add(a, b)
    torch.testing.assert_close(c, a + b, rtol=0, atol=0)
    assert hk.diag_vector_add(0, 50000) < 1e-6


@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (256, 384, 512), (1000, 520, 264), (4096, 4096, 4096), (33, 17, 8)])
def test_gemm_bf16_nt_matches_fp32_reference(hk, M, N, K):
    torch.manual_seed(0)
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    ref = a.float() @ b.float().T
    out = hk.gemm_bf16_nt(a, b, out_fp32=True)
    torch.testing.assert_close(out, ref, rtol=2e-3, atol=2e-3 * (K ** 0.5))
    outb = hk.gemm_bf16_nt(a, b, out_fp32=False)
    torch.testing.assert_close(outb.float(), ref, rtol=2e-2, atol=2e-2 * (K ** 0.5))


def test_gemm_identity_asymmetric(hk):
    # A = I with an asymmetric B catches a transposed C write (guide §3)
    n = 128
    a = torch.eye(n, device="cuda", dtype=torch.bfloat16)
    b = (torch.arange(n * n, device="cuda").reshape(n, n) % 7 - 3).to(torch.bfloat16)
    out = hk.gemm_bf16_nt(a, b)
    torch.testing.assert_close(out, b.float().T, rtol=0, atol=0)


def test_diag_mfma_and_hbm(hk):
    r = hk.diag_mfma(0, 4096, 10)
    assert r["max_rel_err"] < 1e-2, r
    assert r["tflops"] > 50, r
    h = hk.diag_hbm(0, 1 << 30, 10)
    assert h["GBps"] > 1000, h


def test_payload(hk):
    p = hk.Payload(0)
    try:
        assert all(p.run() for _ in range(10))
    finally:
        p.close()


def test_real_amdsmi_enumerates_mi355x():
    from kubernetes_amd.native import amdsmi
    smi = amdsmi.SMI()
    assert smi.backend == amdsmi.BACKEND_AMDSMI
    assert smi.count() >= 1
    g = smi.gpu(0)
    print(g, smi.metrics(0))
    assert g.arch.startswith("gfx950"), g
    assert g.product in ("MI355X", "MI350X"), g
    assert g.vram_total_mb > 250_000, g
    assert os.path.exists(f"/dev/dri/renderD{g.render_minor}")


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (256, 256, 128), (512, 512, 192), (512, 768, 1024),
                                   (2048, 1024, 4096), (768, 512, 320)])
def test_gemm_both_paths_match_reference(hk, M, N, K):
    """Every GEMM path against an fp32 torch reference: 0/3 = ping-pong 256-tile (K-tile counts 1,
    2, 3 exercise its unrolled pairs, odd tail and counted-vmcnt waits), 4-6 its variants, 1 =
    128-tile register-staged, 2 = 2-barrier 256-tile glds, 7 = 8-phase 256-tile."""
    torch.manual_seed(1)
    a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    ref = a.float() @ b.float().T
    try:
        for path in (0, 1, 2, 4, 5, 6, 7):
            hk.set_gemm_path(path)
            out = hk.gemm_bf16_nt(a, b, out_fp32=True)
            torch.testing.assert_close(out, ref, rtol=2e-3, atol=2e-3 * (K ** 0.5))
            outb = hk.gemm_bf16_nt(a, b, out_fp32=False).float()
            torch.testing.assert_close(outb, ref, rtol=2e-2, atol=2e-2 * (K ** 0.5))
    finally:
        hk.set_gemm_path(0)


def test_gemm256_identity_asymmetric(hk):
    n = 256
    a = torch.eye(n, device="cuda", dtype=torch.bfloat16)
    b = (torch.arange(n * n, device="cuda").reshape(n, n) % 7 - 3).to(torch.bfloat16)
    torch.testing.assert_close(hk.gemm_bf16_nt(a, b), b.float().T, rtol=0, atol=0)
    torch.testing.assert_close(hk.gemm_bf16_nt(b, a), b.float(), rtol=0, atol=0)


def test_payload_batch(hk):
    """k container starts in one batch: k launches + one verify kernel + one sync, every start verified."""
    p = hk.Payload(0)
    try:
        assert p.run_batch(1) == [True]
        assert p.run_batch(300) == [True] * 300          # > one slot ring: split into batches
        assert all(p.run() for _ in range(3))
    finally:
        p.close()


def _fp8_operands(M, N, K, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    a = (torch.rand(M, K, device="cuda", generator=g) * 4 - 2).to(torch.float8_e4m3fn)
    b = (torch.rand(N, K, device="cuda", generator=g) * 4 - 2).to(torch.float8_e4m3fn)
    return a, b


@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (256, 256, 256), (512, 768, 384), (1024, 512, 2048),
                                   (768, 256, 640)])
def test_gemm_fp8_matches_fp32_reference(hk, M, N, K):
    """fp8 e4m3 x fp8 e4m3 products are exact in fp32, so the only difference from the fp32
    reference of the same (dequantized) operands is the summation order."""
    a, b = _fp8_operands(M, N, K)
    ref = a.float() @ b.float().T
    out = hk.gemm_fp8_nt(a, b)
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-3 * (K ** 0.5))
    out16 = hk.gemm_fp8_nt(a, b, out_fp32=False)
    assert out16.dtype == torch.bfloat16
    torch.testing.assert_close(out16.float(), ref, rtol=1e-2, atol=1e-2 * (K ** 0.5))


def test_gemm_fp8_identity_asymmetric(hk):
    """A = I with an asymmetric B catches a row/col swap and any A/B k-slot mispairing."""
    n = 256
    eye = torch.eye(n, device="cuda").to(torch.float8_e4m3fn)
    b = (torch.arange(n * n, device="cuda").reshape(n, n) % 7 - 3).float().to(torch.float8_e4m3fn)
    torch.testing.assert_close(hk.gemm_fp8_nt(eye, b), b.float().T, rtol=0, atol=0)
    torch.testing.assert_close(hk.gemm_fp8_nt(b, eye), b.float(), rtol=0, atol=0)


def test_gemm_fp8_rejects_untiled_shapes(hk):
    a, b = _fp8_operands(256, 256, 128)
    with pytest.raises(ValueError):
        hk.gemm_fp8_nt(a[:, :64].contiguous(), b[:, :64].contiguous())


def test_diag_mfma_fp8(hk):
    r = hk.diag_mfma_fp8(0, 4096, 5)
    print(r)
    assert r["max_rel_err"] < 1e-5 and r["tflops"] > 500
