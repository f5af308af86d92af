"""The large-tile decode GEMM with everything between the GEMMs folded in
(csrc/tgemm.hip TgEpi, round 6): split-K reduced inside the GEMM by the last
arriving block of each (weight tile, M part) -- no reduction kernel -- and
each RMSNorm applied as the next GEMM's per-row factor from the row sums of
squares the residual-writing GEMM leaves.  Every mode against plain PyTorch
fp32 compositions of the same ops, at the row counts of the > 512-row decode
steps, for several split counts (the fixup's ticket reset and cross-launch
slab reuse included: back-to-back launches on changing inputs)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

ROWS = [513, 610, 768, 1024]


@pytest.fixture(scope="module")
def hip():
    from dmcp.ops import hip as h
    h.lib()
    return h


@pytest.fixture(scope="module")
def ws(hip):
    return hip.tgemm_fixup_workspace(1024, 3072, 2048, "cuda")


def _bf(*shape, seed=0, scale=1.0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return (torch.randn(*shape, generator=g, device="cuda") * scale).to(torch.bfloat16)


def _rs_ref(x, eps):
    x = x.float()
    return torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps)


@pytest.mark.parametrize("M", ROWS)
@pytest.mark.parametrize("K,S", [(2048, 1), (2048, 2), (2048, 3), (8192, 6), (8192, 11)])
def test_tgemm_resid_fixup(hip, ws, M, K, S):
    N, eps = 2048, 1e-5
    x, w = _bf(M, K, seed=1 + S), _bf(N, K, seed=2, scale=0.02)
    resid = _bf(M, N, seed=3)
    r_exp = (resid.float() + (x.float() @ w.float().t()).to(torch.bfloat16).float()).to(torch.bfloat16)
    got = resid.clone()
    rs = hip.tgemm_resid(x, w, got, ws, eps, splits=S)
    torch.testing.assert_close(got.float(), r_exp.float(), atol=3e-2, rtol=3e-2)
    sq = r_exp.float().view(M, N // 256, 256).pow(2).sum(-1).t()  # [tiles, M]
    torch.testing.assert_close(rs.sq, sq, atol=1e-2, rtol=2e-3)
    assert rs.n == N and rs.eps == eps
    assert int(ws["cnt"].abs().sum()) == 0  # every ticket reset by its last arriver


@pytest.mark.parametrize("M", [610, 1024])
def test_tgemm_resid_back_to_back_launches(hip, ws, M):
    """Ten launches in one stream on changing inputs and split counts, each
    checked: a stale slab (a last arriver reading another slice's previous
    launch) or a ticket left non-zero shows up as a wrong row."""
    N, K = 2048, 2048
    w = _bf(N, K, seed=5, scale=0.02)
    outs, exps = [], []
    for it in range(10):
        x = _bf(M, K, seed=100 + it)
        resid = _bf(M, N, seed=200 + it)
        exps.append((resid.float() + (x.float() @ w.float().t()).to(torch.bfloat16).float()).to(torch.bfloat16))
        hip.tgemm_resid(x, w, resid, ws, 1e-5, splits=(2, 3, 4, 8)[it % 4], mparts=(0, 5, 10)[it % 3])
        outs.append(resid)
    torch.cuda.synchronize()
    for o, e in zip(outs, exps):
        torch.testing.assert_close(o.float(), e.float(), atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("M", [513, 610, 1024])
@pytest.mark.parametrize("kv", ["bf16", "fp8"])
@pytest.mark.parametrize("S", [1, 2, 4])
@pytest.mark.parametrize("scaled", [False, True])
def test_tgemm_qkv_fixup(hip, ws, M, kv, S, scaled):
    from dmcp.ops import reference
    from dmcp.ops.reference import kv_float
    Hq, Hkv, D, K, MAXS, NS = 32, 8, 64, 2048, 512, 6
    N, eps = (Hq + 2 * Hkv) * D, 1e-5
    x, w = _bf(M, K, seed=11), _bf(N, K, seed=12, scale=0.05)
    dt = torch.uint8 if kv == "fp8" else torch.bfloat16
    kc = torch.zeros((NS, Hkv, MAXS, D), dtype=dt, device="cuda")
    vc = torch.zeros_like(kc)
    kr, vr = kc.clone(), vc.clone()
    pos = torch.tensor([m // NS for m in range(M)], dtype=torch.int32, device="cuda")
    slot = torch.tensor([m % NS if m % 11 else -1 for m in range(M)], dtype=torch.int32, device="cuda")
    cs = reference.rope_tables(MAXS, D, 10000.0, device="cuda")
    rs = None
    xin = x.float()
    if scaled:  # x is an un-normalised residual: the GEMM applies its RMSNorm per row
        sq = x.float().view(M, K // 256, 256).pow(2).sum(-1).t().contiguous()
        rs = hip.RowScale(sq, K, eps)
        xin = (x.float() * _rs_ref(x, eps)).to(torch.bfloat16).float()
    q = hip.tgemm_qkv(x, w, pos, slot, cs, kc, vc, Hq, ws, row_scale=rs, splits=S)
    qkv = (xin @ w.float().t()).to(torch.bfloat16)
    qr = reference.rope_kv(qkv, pos, slot, cs, kr, vr, Hq)
    torch.testing.assert_close(q.float(), qr.float(), atol=4e-2, rtol=4e-2)
    tol = dict(atol=4e-2, rtol=0.13) if kv == "fp8" else dict(atol=4e-2, rtol=4e-2)
    torch.testing.assert_close(kv_float(kc), kv_float(kr), **tol)
    torch.testing.assert_close(kv_float(vc), kv_float(vr), **tol)
    assert int(ws["cnt"].abs().sum()) == 0


@pytest.mark.parametrize("M", ROWS)
def test_tgemm_swiglu_row_scale(hip, M):
    K, inter, eps = 2048, 8192, 1e-5
    x, w = _bf(M, K, seed=31, scale=3.0), _bf(2 * inter, K, seed=32, scale=0.05)
    sq = x.float().view(M, K // 256, 256).pow(2).sum(-1).t().contiguous()
    got = hip.tgemm_swiglu_scaled(x, w, hip.RowScale(sq, K, eps))
    h = (x.float() * _rs_ref(x, eps)).to(torch.bfloat16).float()
    gu = (h @ w.float().t()).to(torch.bfloat16).float()
    exp = torch.nn.functional.silu(gu[:, :inter]) * gu[:, inter:]
    torch.testing.assert_close(got.float(), exp, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("M", [610, 1024])
def test_tgemm_head_row_scale_selects_the_normalised_argmax(hip, M):
    V, K, eps = 128256, 2048, 1e-5
    g = torch.Generator().manual_seed(M)
    x = (torch.randn(M, K, generator=g) * 4).to(torch.bfloat16).cuda()
    w = (torch.randn(V, K, generator=g) * 0.02).to(torch.bfloat16).cuda()
    masks = torch.full((1, (V + 31) // 32), -1, dtype=torch.int32, device="cuda")
    midx = torch.zeros(M, dtype=torch.int32, device="cuda")
    sq = x.float().view(M, K // 256, 256).pow(2).sum(-1).t().contiguous()
    ids = hip.tgemm_lm_head_argmax(x, w, masks, midx, row_scale=hip.RowScale(sq, K, eps)).cpu().long()
    ref = ((x.float() * _rs_ref(x, eps)) @ w.float().t()).cpu()
    best = ref.max(1).values
    picked = ref.gather(1, ids[:, None])[:, 0]
    assert bool((picked >= best - 1e-2 * best.abs().clamp_min(1.0)).all())
    assert (ids == ref.argmax(1)).float().mean() > 0.97


def test_fixup_validation(hip, ws):
    with pytest.raises(hip.HipOpsError):  # head_dim 128
        hip.tgemm_qkv(_bf(600, 2048), _bf(4096, 2048), torch.zeros(600, dtype=torch.int32, device="cuda"),
                      torch.zeros(600, dtype=torch.int32, device="cuda"),
                      torch.zeros((64, 64, 2), device="cuda"),
                      torch.zeros((2, 8, 64, 128), dtype=torch.bfloat16, device="cuda"),
                      torch.zeros((2, 8, 64, 128), dtype=torch.bfloat16, device="cuda"), 16, ws)
    with pytest.raises(hip.HipOpsError):  # residual shape
        hip.tgemm_resid(_bf(600, 2048), _bf(2048, 2048), _bf(600, 1024), ws, 1e-5)
    with pytest.raises(hip.HipOpsError):  # a row scale of the wrong row count
        hip.tgemm_swiglu_scaled(_bf(600, 2048), _bf(1024, 2048),
                                hip.RowScale(torch.ones((8, 500), device="cuda"), 2048, 1e-5))


@pytest.fixture(scope="module")
def llama_like():
    """Llama-3.2-1B layer geometry (hidden 2048, 32 / 8 heads of 64,
    intermediate 8192) over 2 layers and a 512-id vocabulary, with
    non-trivial norm weights (folded into the matrices at load)."""
    from dmcp.models.llm import LocalLM, LMConfig
    cfg = LMConfig(name="llama-like", vocab_size=512, hidden=2048, layers=2, n_heads=32, n_kv_heads=8, head_dim=64,
                   intermediate=8192, max_seq=512, max_batch=64, max_rows=1024, kv_dtype="fp8")
    m = LocalLM(cfg, device="cuda", seed=5)
    g = torch.Generator(device="cuda").manual_seed(9)
    w = {k: v.clone() for k, v in m.w.items()}
    for k in list(w):
        if k.endswith(("ln1", "ln2")) or k == "norm_f":
            w[k] = (1 + 0.3 * torch.randn(cfg.hidden, generator=g, device="cuda")).to(torch.bfloat16)
    return LocalLM(cfg, device="cuda", weights=w)


@pytest.mark.parametrize("rows", [513, 610, 768, 1024])
def test_model_fixup_trunk_matches_the_reduction_kernel_trunk(llama_like, rows):
    """A > 512-row step on the fixup trunk == the same step on the round-5
    trunk (split-K partials + reduction kernels + norm passes), and row 0
    tracks the fp32 reference model."""
    m = llama_like
    assert m.tg_fixup
    toks = [256] + list(b"@Service class OrderService {")
    for s in range(64):
        m.forward_tokens(torch.tensor(toks, dtype=torch.int32), s, 0)
    tk = torch.tensor([ord("a") + (r % 20) for r in range(rows)], dtype=torch.int32, device="cuda")
    sl = torch.tensor([r % 64 for r in range(rows)], dtype=torch.int32, device="cuda")
    ps = torch.tensor([len(toks) + r // 64 for r in range(rows)], dtype=torch.int32, device="cuda")
    m.tg_fixup = False
    try:
        ref = m.decode(tk, sl, ps).float()
    finally:
        m.tg_fixup = True
    got = m.decode(tk, sl, ps).float()
    err = (got - ref).abs().max().item() / max(1.0, ref.abs().max().item())
    assert err < 0.03, err
    exp = m.reference_logits(toks + [int(tk[0])])[-1].float()
    assert (got[0] - exp).abs().max().item() / max(1.0, exp.abs().max().item()) < 0.05
    cos = torch.nn.functional.cosine_similarity(got[0], exp, dim=0).item()
    assert cos > 0.999, cos
