"""Fused decode GEMMs (csrc/fused_gemm.hip) against plain PyTorch fp32
compositions of the same ops, and the fused decode step against the
hipBLASLt + element-wise-kernel step and the fp32 reference model."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hip():
    from dmcp.ops import hip as h
    h.lib()
    return h


def _bf(*shape, seed=0, scale=1.0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return (torch.randn(*shape, generator=g, device="cuda") * scale).to(torch.bfloat16)


def _rms(x, eps):
    x = x.float()
    return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps)


ROWS = [1, 5, 16, 33, 78, 96, 128]


@pytest.mark.parametrize("M", ROWS)
def test_fused_linear_norm(hip, M):
    K, N, eps = 512, 320, 1e-5
    x, w = _bf(M, K, seed=1), _bf(N, K, seed=2, scale=0.05)
    got = hip.fused_linear_norm(x, w, eps)
    exp = _rms(x, eps) @ w.float().t()
    torch.testing.assert_close(got.float(), exp, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("M", ROWS)
@pytest.mark.parametrize("K", [512, 2048, 8192])
def test_fused_resid(hip, M, K):
    N = 256
    x, w = _bf(M, K, seed=3), _bf(N, K, seed=4, scale=0.02)
    r = _bf(M, N, seed=5)
    exp = r.float() + x.float() @ w.float().t()
    got = hip.fused_resid(x, w, r.clone(), wk=16 if K >= 4096 else 8)
    torch.testing.assert_close(got.float(), exp, atol=4e-2, rtol=2e-2)


@pytest.mark.parametrize("M", ROWS)
def test_fused_swiglu(hip, M):
    K, inter, eps = 1024, 512, 1e-5
    x, w = _bf(M, K, seed=6), _bf(2 * inter, K, seed=7, scale=0.05)
    got = hip.fused_swiglu(x, w, eps)
    gu = _rms(x, eps) @ w.float().t()
    exp = torch.nn.functional.silu(gu[:, :inter]) * gu[:, inter:]
    torch.testing.assert_close(got.float(), exp, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("D,Hq,Hkv", [(64, 32, 8), (128, 8, 2), (64, 4, 2)])
@pytest.mark.parametrize("M", [1, 7, 78, 128])
def test_fused_rope_kv(hip, D, Hq, Hkv, M):
    from dmcp.ops import reference
    K, S, MAXS, eps = 512, 6, 256, 1e-5
    x, w = _bf(M, K, seed=8), _bf((Hq + 2 * Hkv) * D, K, seed=9, scale=0.05)
    slot = torch.tensor([m % S for m in range(M)], dtype=torch.int32, device="cuda")
    if M > 1:
        slot[M // 2] = -1  # padding row: no cache write
    # distinct (slot, pos) per row so the reference cache is unambiguous
    pos = torch.tensor([(m // S) * 3 + 1 for m in range(M)], dtype=torch.int32, device="cuda")
    cs = reference.rope_tables(MAXS, D, device="cuda")
    kc = torch.zeros(S, Hkv, MAXS, D, dtype=torch.bfloat16, device="cuda")
    vc = torch.zeros_like(kc)
    q = hip.fused_rope_kv(x, w, eps, pos, slot, cs, kc, vc, Hq)
    qkv = (_rms(x, eps) @ w.float().t())
    kr = torch.zeros(S, Hkv, MAXS, D, dtype=torch.float32, device="cuda")
    vr = torch.zeros_like(kr)
    qr = reference.rope_kv(qkv, pos, slot, cs, kr, vr, Hq)
    torch.testing.assert_close(q.float(), qr.float(), atol=3e-2, rtol=3e-2)
    torch.testing.assert_close(kc.float(), kr, atol=3e-2, rtol=3e-2)
    torch.testing.assert_close(vc.float(), vr, atol=3e-2, rtol=3e-2)


def test_fused_shape_validation(hip):
    with pytest.raises(hip.HipOpsError):  # too many rows for the fused path
        hip.fused_linear_norm(_bf(129, 64), _bf(64, 64), 1e-5)
    with pytest.raises(hip.HipOpsError):  # K not a multiple of 32
        hip.fused_resid(_bf(4, 48), _bf(64, 48), _bf(4, 64))
    with pytest.raises(hip.HipOpsError):  # residual of the wrong shape
        hip.fused_resid(_bf(4, 64), _bf(64, 64), _bf(3, 64))
    with pytest.raises(hip.HipOpsError):  # undersized output buffer
        hip.fused_swiglu(_bf(4, 64), _bf(64, 64), 1e-5, out=_bf(4, 16))


@pytest.fixture(scope="module")
def model():
    from dmcp.models.llm import LocalLM, preset
    return LocalLM(preset("tiny", max_batch=16), device="cuda", seed=3)


@pytest.mark.parametrize("rows", [1, 9, 40])
def test_fused_decode_matches_unfused_and_reference(model, rows):
    """The fused decode step == the hipBLASLt + element-wise-kernel step (and
    the fp32 reference for row 0) on rows extending several slots."""
    toks = [256] + list(b"@RestController class OrderController {")
    for s in range(4):
        model.forward_tokens(torch.tensor(toks, dtype=torch.int32), s, 0)
    tk = torch.tensor([ord("a") + (r % 20) for r in range(rows)], dtype=torch.int32, device="cuda")
    sl = torch.tensor([r % 4 for r in range(rows)], dtype=torch.int32, device="cuda")
    ps = torch.tensor([len(toks) + r // 4 for r in range(rows)], dtype=torch.int32, device="cuda")
    model.use_fused = False
    ref = model.decode(tk, sl, ps).float()
    model.use_fused, model.fused_max_rows = True, 128
    got = model.decode(tk, sl, ps).float()
    err = (got - ref).abs().max().item() / max(1.0, ref.abs().max().item())
    assert err < 0.03, err
    if rows == 1:
        exp = model.reference_logits(toks + [int(tk[0])])[-1].float()
        assert (got[0] - exp).abs().max().item() / max(1.0, exp.abs().max().item()) < 0.03


def test_fold_norms_preserves_the_model():
    """Loading a checkpoint with non-trivial norm weights folds them into the
    consumer matrices; logits are unchanged (fp32 reference)."""
    from dmcp.models.llm import LocalLM, preset
    cfg = preset("tiny", max_batch=2)
    base = LocalLM(cfg, device="cuda", seed=4)
    w = {k: v.clone() for k, v in base.w.items()}
    g = torch.Generator(device="cuda").manual_seed(0)
    for k in list(w):
        if k.endswith(("ln1", "ln2")) or k == "norm_f":
            w[k] = (1 + 0.3 * torch.randn(w[k].shape, generator=g, device="cuda")).to(torch.bfloat16)
    unfolded = {k: v.float() for k, v in w.items()}
    m = LocalLM(cfg, device="cuda", weights=dict(w))
    assert all(bool((m.w[k] == 1).all()) for k in m.w if k.endswith(("ln1", "ln2")) or k == "norm_f")
    toks = [256] + list(b"class A {}")
    got = m.reference_logits(toks)[-1]
    # the unfolded model, computed directly
    c = cfg
    x = unfolded["embed"][torch.tensor(toks, device="cuda")]
    T = len(toks)

    def rms(t, gw):
        return t * torch.rsqrt(t.pow(2).mean(-1, keepdim=True) + c.eps) * gw
    from dmcp.ops import reference
    cs = m.cos_sin
    pos = torch.arange(T, device="cuda", dtype=torch.int32)
    G = c.n_heads // c.n_kv_heads
    for i in range(c.layers):
        h = rms(x, unfolded[f"l{i}.ln1"])
        qkv = (h @ unfolded[f"l{i}.wqkv"].t()).view(T, c.n_heads + 2 * c.n_kv_heads, c.head_dim)
        q = reference.apply_rope(qkv[:, :c.n_heads], pos, cs)
        k = reference.apply_rope(qkv[:, c.n_heads:c.n_heads + c.n_kv_heads], pos, cs).repeat_interleave(G, 1)
        v = qkv[:, c.n_heads + c.n_kv_heads:].repeat_interleave(G, 1)
        att = torch.einsum("thd,shd->hts", q, k) / math.sqrt(c.head_dim)
        att = att.masked_fill(torch.triu(torch.ones(T, T, dtype=torch.bool, device="cuda"), 1), float("-inf"))
        x = x + torch.einsum("hts,shd->thd", att.softmax(-1), v).reshape(T, -1) @ unfolded[f"l{i}.wo"].t()
        gu = rms(x, unfolded[f"l{i}.ln2"]) @ unfolded[f"l{i}.wgu"].t()
        x = x + (torch.nn.functional.silu(gu[:, :c.intermediate]) * gu[:, c.intermediate:]) @ \
            unfolded[f"l{i}.wdown"].t()
    exp = (rms(x, unfolded["norm_f"]) @ unfolded["lm_head"].t())[-1]
    assert (got - exp).abs().max().item() / max(1.0, exp.abs().max().item()) < 0.03


def test_odd_vocab_checkpoint_decodes_on_the_library_path():
    """A vocab outside the fused kernels' contract (e.g. 32001-style sizes)
    disables the fused path at init instead of failing on small steps."""
    from dmcp.models.llm import LocalLM, fused_shapes_ok, preset
    cfg = preset("tiny", max_batch=4, vocab_size=321)
    assert not fused_shapes_ok(cfg)
    m = LocalLM(cfg, device="cuda", seed=5)
    assert not m.use_fused
    toks = [256] + list(b"class A {")
    m.forward_tokens(torch.tensor(toks, dtype=torch.int32), 0, 0)
    got = m.decode(torch.tensor([ord("x")], dtype=torch.int32, device="cuda"),
                   torch.tensor([0], dtype=torch.int32, device="cuda"),
                   torch.tensor([len(toks)], dtype=torch.int32, device="cuda")).float()[0]
    exp = m.reference_logits(toks + [ord("x")])[-1].float()
    assert got.shape[0] == 321
    assert (got - exp).abs().max().item() / max(1.0, exp.abs().max().item()) < 0.03
