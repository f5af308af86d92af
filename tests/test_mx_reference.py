"""CPU checks of the MXFP8 reference ops (dmcp.ops.reference): the block
quantiser's error bound and exponent rule, weight quantisation, and the
prefill GEMM compositions the GPU kernels are tested against."""
import torch

from dmcp.ops import reference as R


def test_mx_quant_error_bound_and_exponents():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(64, 256, generator=g) * torch.logspace(-3, 3, 64)[:, None]
    x[3, :32] = 0
    q, s = R.mx_quant(x)
    assert q.dtype == torch.uint8 and q.shape == x.shape and s.shape == (64, 8)
    back = R.mx_dequant(q, s)
    blk = x.abs().reshape(64, 8, 32).amax(-1)
    # the block's largest value maps into (224, 448]: e4m3 keeps 3 mantissa bits
    assert ((back - x).abs().reshape(64, 8, 32) <= blk[..., None] / 16 + 1e-30).all()
    e = s.to(torch.int32) - 127
    nz = blk > 0
    assert (blk[nz] / 2.0 ** e[nz].float() <= 448).all() and (blk[nz] / 2.0 ** e[nz].float() > 224).all()
    assert (back[3, :32] == 0).all()


def test_quantize_weight_per_row():
    g = torch.Generator().manual_seed(1)
    w = torch.randn(96, 128, generator=g) * torch.linspace(0.01, 2, 96)[:, None]
    w[5] = 0
    wq, ws = R.quantize_weight(w)
    assert wq.dtype == torch.uint8 and ws.dtype == torch.float32 and ws.shape == (96,)
    back = R.weight_dequant(wq, ws)
    assert ((back - w).abs() <= w.abs().amax(-1, keepdim=True) / 16 + 1e-12).all()
    assert ws[5] == 1 and (back[5] == 0).all()


def test_pgemm_compositions_close_to_bf16():
    g = torch.Generator().manual_seed(2)
    M, K, N = 40, 256, 512
    x = torch.randn(M, K, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.05).to(torch.bfloat16)
    aq, as_ = R.mx_quant(x)
    wq, ws = R.quantize_weight(w)
    y = R.pgemm(aq, as_, wq, ws)
    exact = x.float() @ w.float().t()
    rel = (y.float() - exact).norm() / exact.norm()
    assert rel < 0.06, rel
    resid = torch.zeros(M, N, dtype=torch.bfloat16)
    R.pgemm_resid(aq, as_, wq, ws, resid)
    assert torch.equal(resid, y)
    q, s = R.pgemm_swiglu(aq, as_, wq, ws)
    assert q.shape == (M, N // 2) and s.shape == (M, N // 64)
    gg, uu = y.float()[:, :N // 2], y.float()[:, N // 2:]
    act = gg / (1 + torch.exp(-gg)) * uu
    assert (R.mx_dequant(q, s) - act).norm() / act.norm() < 0.06


def test_rmsnorm_mx_updates_residual():
    g = torch.Generator().manual_seed(3)
    resid = torch.randn(4, 2048, generator=g).to(torch.bfloat16)
    add = torch.randn(4, 2048, generator=g).to(torch.bfloat16)
    w = torch.ones(2048, dtype=torch.bfloat16)
    before = resid.clone()
    q, s = R.rmsnorm_mx(resid, w, 1e-5, add=add)
    assert torch.equal(resid, (before.float() + add.float()).to(torch.bfloat16))
    h = resid.float() * torch.rsqrt(resid.float().pow(2).mean(-1, keepdim=True) + 1e-5)
    assert (R.mx_dequant(q, s) - h).norm() / h.norm() < 0.06
