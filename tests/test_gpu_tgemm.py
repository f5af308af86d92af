"""Large-tile decode GEMM (csrc/tgemm.hip) against plain PyTorch fp32
compositions of the same ops at the row counts of large decode steps
(257-1024: the engine's max_rows is 768 at 512 KV slots), for every epilogue:
bf16 output, split-K partials (uneven slice counts included), SwiGLU,
residual + RMSNorm and RoPE + KV-cache append (through wgemm.hip's fused
reductions), and the LM head + grammar-masked argmax."""
import pytest
import torch

pytestmark = pytest.mark.gpu

ROWS = [257, 513, 600, 768, 1024]


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


@pytest.mark.parametrize("M", ROWS + [1, 40])
@pytest.mark.parametrize("N,K", [(3072, 2048), (2048, 8192), (512, 384)])
def test_tgemm_plain(hip, M, N, K):
    x, w = _bf(M, K, seed=1), _bf(N, K, seed=2, scale=0.05)
    got = hip.tgemm(x, w)
    exp = x.float() @ w.float().t()
    torch.testing.assert_close(got.float(), exp, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("M", ROWS)
@pytest.mark.parametrize("S", [1, 3, 7, 8])
def test_tgemm_partials_sum_to_the_product(hip, M, S):
    N, K = 2048, 2048
    x, w = _bf(M, K, seed=3), _bf(N, K, seed=4, scale=0.05)
    ws = torch.full((16 * M * N,), float("nan"), dtype=torch.float32, device="cuda")
    got = hip.tgemm_partials(x, w, ws, splits=S)
    assert got == S
    total = ws[:S * M * N].view(S, M, N).sum(0)
    torch.testing.assert_close(total, x.float() @ w.float().t(), atol=1e-2, rtol=1e-2)


@pytest.mark.parametrize("M", ROWS)
@pytest.mark.parametrize("mparts", [0, 4, 8])
def test_tgemm_every_m_split(hip, M, mparts):
    """Any M-part count whose parts stay <= 256 rows (the plan's choice and
    forced ones) covers every row exactly."""
    if mparts and -(-M // mparts) > 256:
        pytest.skip("parts over 256 rows")
    N, K = 1024, 512
    x, w = _bf(M, K, seed=21), _bf(N, K, seed=22, scale=0.05)
    out = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device="cuda")
    hip.tgemm(x, w, out=out, mparts=mparts)
    torch.testing.assert_close(out.float(), x.float() @ w.float().t(), atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("M", ROWS)
@pytest.mark.parametrize("inter", [1024, 8192])
def test_tgemm_swiglu(hip, M, inter):
    K = 2048
    x, w = _bf(M, K, seed=5), _bf(2 * inter, K, seed=6, scale=0.05)
    got = hip.tgemm_swiglu(x, w)
    gu = (x.float() @ w.float().t()).to(torch.bfloat16).float()
    exp = torch.nn.functional.silu(gu[:, :inter]) * gu[:, inter:]
    assert got.shape == (M, inter)
    torch.testing.assert_close(got.float(), exp, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("M", ROWS)
@pytest.mark.parametrize("N,K", [(2048, 2048), (2048, 8192)])
def test_tgemm_resid_norm(hip, M, N, K):
    eps = 1e-5
    x, w = _bf(M, K, seed=7), _bf(N, K, seed=8, scale=0.02)
    resid = _bf(M, N, seed=9)
    g = (1 + 0.1 * torch.randn(N, generator=torch.Generator(device="cuda").manual_seed(10),
                               device="cuda")).to(torch.bfloat16)
    r_exp = (resid.float() + (x.float() @ w.float().t()).to(torch.bfloat16).float()).to(torch.bfloat16)
    exp = _rms(r_exp, eps) * g.float()
    ws = torch.empty(16 * M * N, dtype=torch.float32, device="cuda")
    r_got = resid.clone()
    got = hip.tgemm_resid_norm(x, w, r_got, g, eps, ws)
    torch.testing.assert_close(r_got.float(), r_exp.float(), atol=3e-2, rtol=3e-2)
    torch.testing.assert_close(got.float(), exp, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("M", [257, 600, 1024])
@pytest.mark.parametrize("kv", ["bf16", "fp8"])
def test_tgemm_rope_kv(hip, M, kv):
    from dmcp.ops import reference
    Hq, Hkv, D, K, MAXS, S = 32, 8, 64, 2048, 512, 6
    N = (Hq + 2 * Hkv) * D
    x, w = _bf(M, K, seed=11), _bf(N, K, seed=12, scale=0.05)
    dt = torch.uint8 if kv == "fp8" else torch.bfloat16
    kc = torch.zeros((S, Hkv, MAXS, D), dtype=dt, device="cuda")
    vc = torch.zeros_like(kc)
    kr, vr = kc.clone(), vc.clone()
    # one (slot, position) per row: rows never write the same cache entry
    pos = torch.tensor([m // S for m in range(M)], dtype=torch.int32, device="cuda")
    slot = torch.tensor([m % S if m % 11 else -1 for m in range(M)], dtype=torch.int32, device="cuda")
    cs = reference.rope_tables(MAXS, D, 10000.0, device="cuda")
    ws = torch.empty(16 * M * N, dtype=torch.float32, device="cuda")
    q = hip.tgemm_rope_kv(x, w, pos, slot, cs, kc, vc, Hq, ws)
    qkv = (x.float() @ w.float().t()).to(torch.bfloat16)
    qr = reference.rope_kv(qkv, pos, slot, cs, kr, vr, Hq)
    torch.testing.assert_close(q.float(), qr.float(), atol=3e-2, rtol=3e-2)
    from dmcp.ops.reference import kv_float
    tol = dict(atol=3e-2, rtol=0.13) if kv == "fp8" else dict(atol=3e-2, rtol=3e-2)
    torch.testing.assert_close(kv_float(kc), kv_float(kr), **tol)
    torch.testing.assert_close(kv_float(vc), kv_float(vr), **tol)


@pytest.mark.parametrize("V", [32000 - 32000 % 256, 128256])
@pytest.mark.parametrize("M", [1, 300, 610, 768, 1024])
def test_tgemm_lm_head_argmax_matches_fp32_reference(hip, V, M):
    """Every selected id is allowed by its row's mask and its fp32 logit is
    the row's masked maximum up to bf16 rounding; nothing allowed -> id 0."""
    K = 2048
    g = torch.Generator().manual_seed(V + M)
    x = (torch.randn(M, K, generator=g) * 0.5).to(torch.bfloat16).cuda()
    w = (torch.randn(V, K, generator=g) * 0.02).to(torch.bfloat16).cuda()
    W = (V + 31) // 32
    dense = torch.randint(-2**31, 2**31 - 1, (3, W), generator=g, dtype=torch.int64).to(torch.int32)
    sp = torch.zeros(1, W, dtype=torch.int64)
    for v in torch.randint(0, V, (40,), generator=g).tolist():
        sp[0, v >> 5] |= 1 << (v & 31)
    sparse = torch.where(sp >= 2**31, sp - 2**32, sp).to(torch.int32)
    masks = torch.cat([dense, sparse, torch.zeros(1, W, dtype=torch.int32)]).cuda()
    midx = torch.randint(0, 5, (M,), generator=g, dtype=torch.int32).cuda()
    ids = hip.tgemm_lm_head_argmax(x, w, masks, midx)
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
    assert exact.float().mean() > 0.97


def test_tgemm_shape_validation(hip):
    with pytest.raises(hip.HipOpsError):  # too many rows
        hip.tgemm(_bf(1025, 64), _bf(256, 64))
    with pytest.raises(hip.HipOpsError):  # K not a multiple of 64
        hip.tgemm(_bf(4, 96), _bf(256, 96))
    with pytest.raises(hip.HipOpsError):  # N not a multiple of 256
        hip.tgemm(_bf(4, 64), _bf(320, 64))
    with pytest.raises(hip.HipOpsError):  # an empty K slice
        hip.tgemm_partials(_bf(600, 128), _bf(256, 128), torch.empty(8 * 600 * 256, dtype=torch.float32,
                                                                        device="cuda"), splits=3)
    with pytest.raises(hip.HipOpsError):  # workspace too small
        hip.tgemm_resid_norm(_bf(600, 2048), _bf(2048, 2048), _bf(600, 2048), _bf(2048), 1e-5,
                             torch.empty(10, dtype=torch.float32, device="cuda"))


@pytest.fixture(scope="module")
def big_model():
    from dmcp.models.llm import LocalLM, preset
    return LocalLM(preset("tiny", max_batch=64, max_rows=1024, max_seq=512), device="cuda", seed=3)


@pytest.mark.parametrize("rows", [513, 700, 1024])
def test_model_decode_on_tgemm_matches_library_path(big_model, rows):
    """A > 512-row decode step on the large-tile GEMMs (+ fused RoPE / KV,
    residual / RMSNorm, SwiGLU) == the same step on hipBLASLt + the unfused
    ops, and row 0 tracks the fp32 reference model."""
    model = big_model
    assert model.use_tgemm
    toks = [256] + list(b"@RestController class OrderController {")
    for s in range(64):
        model.forward_tokens(torch.tensor(toks, dtype=torch.int32), s, 0)
    tk = torch.tensor([ord("a") + (r % 20) for r in range(rows)], dtype=torch.int32, device="cuda")
    sl = torch.tensor([r % 64 for r in range(rows)], dtype=torch.int32, device="cuda")
    ps = torch.tensor([len(toks) + r // 64 for r in range(rows)], dtype=torch.int32, device="cuda")
    model.use_tgemm = False
    ref = model.decode(tk, sl, ps).float()
    model.use_tgemm = True
    got = model.decode(tk, sl, ps).float()
    err = (got - ref).abs().max().item() / max(1.0, ref.abs().max().item())
    assert err < 0.03, err
    exp = model.reference_logits(toks + [int(tk[0])])[-1].float()
    assert (got[0] - exp).abs().max().item() / max(1.0, exp.abs().max().item()) < 0.05


def test_tgemm_head_inside_the_decode_step_matches_the_unfused_head():
    """A > 512-row decode_select_gather of the 128,256-id vocabulary selects
    with the large-tile LM head + masked argmax: the same ids as F.linear +
    masked_argmax on the same trunk (up to near-ties)."""
    from dmcp.enrich.local import LocalEngine
    from dmcp.enrich.tokenizer import load_asset_tokenizer
    from dmcp.models.llm import LocalLM, preset
    m = LocalLM(preset("tiny-bpe", max_batch=64, max_rows=768, max_seq=512), device="cuda:0", seed=2)
    assert m.tg_head and m.tg_head_ws is not None
    masks = LocalEngine(m, use_graphs=False, tokenizer=load_asset_tokenizer(m.cfg.tokenizer)).masks
    B = 600
    for s in range(64):
        m.forward_tokens(torch.tensor([128000, 65 + s % 20, 66], dtype=torch.int32), s, 0)
    tok = torch.randint(32, 120, (B,), dtype=torch.int32).cuda()
    sl = (torch.arange(B, dtype=torch.int32) % 64).cuda()
    ps = (3 + torch.arange(B, dtype=torch.int32) // 64).cuda()
    mi = (torch.arange(B, dtype=torch.int32) % masks.shape[0]).cuda()
    last = torch.zeros(768, dtype=torch.int32).cuda()
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
