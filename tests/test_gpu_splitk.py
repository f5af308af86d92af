"""Split-K decode GEMM with the residual add + RMSNorm folded into its
reduction (csrc/splitk_gemm.hip) against the fp32 reference of
F.linear -> add_rmsnorm (dmcp.ops.reference)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hip():
    from dmcp.ops import hip as h
    h.lib()
    return h


def _bf(*shape, scale=1.0, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return (torch.randn(*shape, generator=g, device="cuda") * scale).to(torch.bfloat16)


@pytest.mark.parametrize("M", [1, 17, 33, 78, 96, 128])
@pytest.mark.parametrize("N,K", [(2048, 2048), (2048, 8192), (512, 1024)])
def test_linear_resid_norm(hip, M, N, K):
    from dmcp.ops import reference
    x = _bf(M, K, seed=M)
    w = _bf(N, K, seed=N + K, scale=0.03)
    resid = _bf(M, N, seed=7)
    g = (1 + 0.1 * _bf(N, seed=8).float()).to(torch.bfloat16)
    S = hip.splitk_splits(N, K)
    ws = torch.empty(S * M * N, dtype=torch.float32, device="cuda")
    r_exp = resid.clone()
    y = (x.float() @ w.float().t()).to(torch.bfloat16)
    exp = reference.add_rmsnorm(y, g, 1e-5, residual=r_exp)
    for variant in (0, 1):
        r_got = resid.clone()
        got = hip.linear_resid_norm(x, w, r_got, g, 1e-5, ws, variant=variant)
        torch.testing.assert_close(r_got.float(), r_exp.float(), atol=3e-2, rtol=2e-2)
        torch.testing.assert_close(got.float(), exp.float(), atol=3e-2, rtol=3e-2)
        for s in (1, 2):  # other split counts give the same result
            r2 = resid.clone()
            torch.testing.assert_close(hip.linear_resid_norm(x, w, r2, g, 1e-5, ws, splits=s, variant=variant).float(),
                                       got.float(), atol=3e-2, rtol=3e-2)


def test_linear_resid_norm_rejects_bad_shapes(hip):
    x, w = _bf(4, 100), _bf(64, 100)
    with pytest.raises(hip.HipOpsError):
        hip.linear_resid_norm(x, w, _bf(4, 64), _bf(64), 1e-5, torch.empty(1 << 16, device="cuda"))
    x, w = _bf(129, 128), _bf(64, 128)
    with pytest.raises(hip.HipOpsError):
        hip.linear_resid_norm(x, w, _bf(129, 64), _bf(64), 1e-5, torch.empty(1 << 20, device="cuda"))


@pytest.mark.parametrize("kv", ["bf16", "fp8"])
@pytest.mark.parametrize("M", [5, 78, 128])
@pytest.mark.parametrize("D,Hq,Hkv", [(64, 32, 8), (128, 16, 8)])
def test_linear_rope_kv(hip, kv, M, D, Hq, Hkv):
    """Split-K QKV + RoPE + cache append == F.linear -> rope_kv (the same
    kernel path the model used before), q and both caches."""
    from dmcp.ops import reference
    K, S, MAXS = 2048, 4, 256
    N = (Hq + 2 * Hkv) * D
    x = _bf(M, K, seed=M + D)
    w = _bf(N, K, seed=3, scale=0.03)
    pos = (torch.arange(M, dtype=torch.int32, device="cuda") * 7) % MAXS
    pos[-1] = -1  # a padding row: q written, caches untouched
    slot = torch.arange(M, dtype=torch.int32, device="cuda") % S
    cs = reference.rope_tables(MAXS, D, device="cuda")
    dt = torch.uint8 if kv == "fp8" else torch.bfloat16
    kc = torch.zeros(S, Hkv, MAXS, D, dtype=dt, device="cuda")
    vc = torch.zeros_like(kc)
    kr, vr = kc.clone(), vc.clone()
    qkv = (x.float() @ w.float().t()).to(torch.bfloat16)
    q_exp = hip.rope_kv(qkv, pos, slot, cs, kr, vr, Hq)
    ws = torch.empty(hip.splitk_splits(N, K) * M * N, dtype=torch.float32, device="cuda")
    for variant in (0, 1):
        kc.zero_()
        vc.zero_()
        q = hip.linear_rope_kv(x, w, pos, slot, cs, kc, vc, Hq, ws, variant=variant)
        torch.testing.assert_close(q.float(), q_exp.float(), atol=3e-2, rtol=2e-2)
        kf, vf = (reference.kv_float(kc), reference.kv_float(vc)) if kv == "fp8" else (kc.float(), vc.float())
        kfr, vfr = (reference.kv_float(kr), reference.kv_float(vr)) if kv == "fp8" else (kr.float(), vr.float())
        tol = dict(atol=3e-2, rtol=0.13) if kv == "fp8" else dict(atol=3e-2, rtol=2e-2)
        torch.testing.assert_close(kf, kfr, **tol)
        torch.testing.assert_close(vf, vfr, **tol)


@pytest.mark.parametrize("M", [3, 78, 128])
def test_linear_resid_norm_swiglu_operand(hip, M):
    """variant 2 reads the gate/up rows and stages silu(gate) * up: equal to
    silu_mul -> linear_resid_norm (and to the fp32 reference)."""
    from dmcp.ops import reference
    N, I = 512, 1024
    gu = _bf(M, 2 * I, seed=M, scale=2.0)
    w = _bf(N, I, seed=9, scale=0.03)
    resid = _bf(M, N, seed=10)
    g = _bf(N, seed=11)
    ws = torch.empty(hip.splitk_splits(N, I) * M * N, dtype=torch.float32, device="cuda")
    act = hip.silu_mul(gu)
    r1, r2 = resid.clone(), resid.clone()
    exp = hip.linear_resid_norm(act, w, r1, g, 1e-5, ws, variant=1)
    got = hip.linear_resid_norm(gu, w, r2, g, 1e-5, ws, variant=2)
    torch.testing.assert_close(got.float(), exp.float(), atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(r2.float(), r1.float(), atol=2e-2, rtol=2e-2)
    r3 = resid.clone()
    y = (reference.silu_mul(gu).float() @ w.float().t()).to(torch.bfloat16)
    ref = reference.add_rmsnorm(y, g, 1e-5, residual=r3)
    torch.testing.assert_close(got.float(), ref.float(), atol=4e-2, rtol=4e-2)
