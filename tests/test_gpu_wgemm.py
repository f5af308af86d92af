"""Weight-streaming decode GEMMs (csrc/wgemm.hip) against plain PyTorch fp32
compositions of the same ops, at the row counts of real decode steps
(17-512: jump-forward steps of 256-512 sequences run 300-500 rows), for every
epilogue: bf16 output, SwiGLU, residual + RMSNorm (split-K reduction), RoPE +
KV-cache append (bf16 and fp8 caches); and the model's decode step on them
against the hipBLASLt path and the fp32 reference model."""
import pytest
import torch

pytestmark = pytest.mark.gpu

ROWS = [17, 33, 78, 129, 256, 320, 384, 448, 512]


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


@pytest.mark.parametrize("M", ROWS)
@pytest.mark.parametrize("N,K", [(3072, 2048), (2048, 8192), (448, 512)])
def test_wgemm_plain(hip, M, N, K):
    x, w = _bf(M, K, seed=1), _bf(N, K, seed=2, scale=0.05)
    got = hip.wgemm(x, w)
    exp = x.float() @ w.float().t()
    torch.testing.assert_close(got.float(), exp, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("M", ROWS)
@pytest.mark.parametrize("S", [2, 4])
def test_wgemm_partials_sum_to_the_product(hip, M, S):
    N, K = 1024, 2048
    x, w = _bf(M, K, seed=3), _bf(N, K, seed=4, scale=0.05)
    ws = torch.empty(8 * M * N, dtype=torch.float32, device="cuda")
    got = hip.wgemm_partials(x, w, ws, splits=S)
    assert got == S
    total = ws[:S * M * N].view(S, M, N).sum(0)
    torch.testing.assert_close(total, x.float() @ w.float().t(), atol=1e-2, rtol=1e-2)


@pytest.mark.parametrize("M", ROWS)
@pytest.mark.parametrize("inter", [1024, 8192])
def test_wgemm_swiglu(hip, M, inter):
    K = 2048
    x, w = _bf(M, K, seed=5), _bf(2 * inter, K, seed=6, scale=0.05)
    got = hip.wgemm_swiglu(x, w)
    gu = (x.float() @ w.float().t()).to(torch.bfloat16).float()
    exp = torch.nn.functional.silu(gu[:, :inter]) * gu[:, inter:]
    assert got.shape == (M, inter)
    torch.testing.assert_close(got.float(), exp, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("M", ROWS)
@pytest.mark.parametrize("N,K", [(2048, 2048), (2048, 8192)])
def test_wgemm_resid_norm(hip, M, N, K):
    eps = 1e-5
    x, w = _bf(M, K, seed=7), _bf(N, K, seed=8, scale=0.02)
    resid = _bf(M, N, seed=9)
    g = (1 + 0.1 * torch.randn(N, generator=torch.Generator(device="cuda").manual_seed(10),
                               device="cuda")).to(torch.bfloat16)
    r_exp = (resid.float() + (x.float() @ w.float().t()).to(torch.bfloat16).float()).to(torch.bfloat16)
    exp = _rms(r_exp, eps) * g.float()
    ws = hip.wgemm_workspace(M, N, "cuda")
    r_got = resid.clone()
    got = hip.wgemm_resid_norm(x, w, r_got, g, eps, ws)
    torch.testing.assert_close(r_got.float(), r_exp.float(), atol=3e-2, rtol=3e-2)
    torch.testing.assert_close(got.float(), exp, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("M", [17, 129, 320])
@pytest.mark.parametrize("kv", ["bf16", "fp8"])
def test_wgemm_rope_kv(hip, M, kv):
    from dmcp.ops import reference
    Hq, Hkv, D, K, MAXS, S = 32, 8, 64, 2048, 512, 6
    N = (Hq + 2 * Hkv) * D
    x, w = _bf(M, K, seed=11), _bf(N, K, seed=12, scale=0.05)
    dt = torch.uint8 if kv == "fp8" else torch.bfloat16
    kc = torch.zeros((S, Hkv, MAXS, D), dtype=dt, device="cuda")
    vc = torch.zeros_like(kc)
    kr, vr = kc.clone(), vc.clone()
    pos = torch.tensor([(7 * m) % MAXS for m in range(M)], dtype=torch.int32, device="cuda")
    slot = torch.tensor([m % S if m % 11 else -1 for m in range(M)], dtype=torch.int32, device="cuda")
    cs = reference.rope_tables(MAXS, D, 10000.0, device="cuda")
    ws = hip.wgemm_workspace(M, N, "cuda")
    q = hip.wgemm_rope_kv(x, w, pos, slot, cs, kc, vc, Hq, ws)
    qkv = (x.float() @ w.float().t()).to(torch.bfloat16)
    qr = reference.rope_kv(qkv, pos, slot, cs, kr, vr, Hq)
    torch.testing.assert_close(q.float(), qr.float(), atol=3e-2, rtol=3e-2)
    from dmcp.ops.reference import kv_float
    tol = dict(atol=3e-2, rtol=0.13) if kv == "fp8" else dict(atol=3e-2, rtol=3e-2)
    torch.testing.assert_close(kv_float(kc), kv_float(kr), **tol)
    torch.testing.assert_close(kv_float(vc), kv_float(vr), **tol)


def test_wgemm_shape_validation(hip):
    with pytest.raises(hip.HipOpsError):  # too many rows
        hip.wgemm(_bf(513, 64), _bf(64, 64))
    with pytest.raises(hip.HipOpsError):  # K not a multiple of 64
        hip.wgemm(_bf(4, 96), _bf(64, 96))
    with pytest.raises(hip.HipOpsError):  # N not a multiple of 64
        hip.wgemm(_bf(4, 64), _bf(80, 64))
    with pytest.raises(hip.HipOpsError):  # workspace too small
        hip.wgemm_resid_norm(_bf(300, 2048), _bf(2048, 2048), _bf(300, 2048), _bf(2048), 1e-5,
                             torch.empty(10, dtype=torch.float32, device="cuda"))


@pytest.fixture(scope="module")
def model():
    from dmcp.models.llm import LocalLM, preset
    return LocalLM(preset("tiny", max_batch=64, max_rows=384, intermediate=1024), device="cuda", seed=3)


@pytest.mark.parametrize("rows", [17, 40, 129, 300])
def test_model_decode_on_wgemm_matches_library_path(model, rows):
    assert model.use_wgemm
    toks = [256] + list(b"@RestController class OrderController {")
    for s in range(8):
        model.forward_tokens(torch.tensor(toks, dtype=torch.int32), s, 0)
    tk = torch.tensor([ord("a") + (r % 20) for r in range(rows)], dtype=torch.int32, device="cuda")
    sl = torch.tensor([r % 8 for r in range(rows)], dtype=torch.int32, device="cuda")
    ps = torch.tensor([len(toks) + r // 8 for r in range(rows)], dtype=torch.int32, device="cuda")
    model.use_wgemm = False
    ref = model.decode(tk, sl, ps).float()
    model.use_wgemm = True
    got = model.decode(tk, sl, ps).float()
    err = (got - ref).abs().max().item() / max(1.0, ref.abs().max().item())
    assert err < 0.03, err
    exp = model.reference_logits(toks + [int(tk[0])])[-1].float()
    assert (got[0] - exp).abs().max().item() / max(1.0, exp.abs().max().item()) < 0.05


@pytest.mark.parametrize("V", [320, 32000, 128256, 151936])
@pytest.mark.parametrize("M", [1, 16, 78, 320, 512, 700])
def test_lm_head_argmax_matches_fp32_reference(V, M):
    """Fused LM head + grammar-masked argmax (no logits written) vs the fp32
    reference: every id is allowed by its row's mask and its fp32 logit is
    the row's masked maximum up to bf16 rounding (ties may resolve to either
    id); a mask row that allows nothing gives id 0, as masked_argmax."""
    from dmcp.ops import hip
    K = 2048 if V >= 32000 else 256
    g = torch.Generator().manual_seed(V + M)
    x = (torch.randn(M, K, generator=g) * 0.5).to(torch.bfloat16).cuda()
    w = (torch.randn(V, K, generator=g) * 0.02).to(torch.bfloat16).cuda()
    W = (V + 31) // 32
    dense = torch.randint(-2**31, 2**31 - 1, (3, W), generator=g, dtype=torch.int64).to(torch.int32)
    sp = torch.zeros(1, W, dtype=torch.int64)
    for v in torch.randint(0, V, (40,), generator=g).tolist():
        sp[0, v >> 5] |= 1 << (v & 31)
    sparse = torch.where(sp >= 2**31, sp - 2**32, sp).to(torch.int32)  # a few allowed ids
    masks = torch.cat([dense, sparse, torch.zeros(1, W, dtype=torch.int32)]).cuda()  # row 4: nothing allowed
    midx = torch.randint(0, 5, (M,), generator=g, dtype=torch.int32).cuda()
    ids = hip.lm_head_argmax(x, w, masks, midx)
    ref = x.float() @ w.float().t()
    bits = ((masks.cpu().long()[midx.cpu().long()][:, torch.arange(V) // 32] >> (torch.arange(V) % 32)) & 1).bool()
    refm = ref.cpu().masked_fill(~bits, float("-inf"))
    best = refm.max(1).values
    got = ids.cpu().long()
    for m in range(M):
        if not bits[m].any():
            assert got[m] == 0
            continue
        assert bits[m, got[m]], f"row {m}: id {got[m]} not allowed"
        assert refm[m, got[m]] >= best[m] - 1e-2 * max(1.0, abs(best[m].item())), f"row {m}"
    exact = (got == refm.argmax(1)) | ~bits.any(1)
    assert exact.float().mean() > 0.97  # only near-ties may differ


def test_lm_head_argmax_inside_the_decode_step_matches_the_unfused_head():
    """decode_select_gather on the fused head == F.linear + masked_argmax
    (the same trunk) for a > 16-row step of the tiny model."""
    from dmcp.enrich.local import LocalEngine
    from dmcp.models.llm import LocalLM, preset
    m = LocalLM(preset("tiny", max_batch=64, max_rows=64, max_seq=512), device="cuda:0", seed=2)
    assert m.fused_head
    masks = LocalEngine(m, use_graphs=False).masks
    B = 40
    for s in range(B):
        m.forward_tokens(torch.tensor([256, 65 + s % 20, 66], dtype=torch.int32), s, 0)
    tok = torch.randint(32, 120, (B,), dtype=torch.int32).cuda()
    sl = torch.arange(B, dtype=torch.int32).cuda()
    ps = torch.full((B,), 3, dtype=torch.int32).cuda()
    mi = (torch.arange(B, dtype=torch.int32) % masks.shape[0]).cuda()
    last = torch.zeros(64, dtype=torch.int32).cuda()
    src = torch.full((B,), -1, dtype=torch.int32).cuda()
    lg, ids = m.decode_select_gather(tok, src, last, sl, ps, masks, mi.clone())
    assert lg is None
    ids = ids.clone()
    m.fused_head = False
    try:
        lg2, ids2 = m.decode_select_gather(tok, src, last, sl, ps, masks, mi.clone())
    finally:
        m.fused_head = True
    assert (ids.cpu() == ids2.cpu()).float().mean() > 0.95
