"""FP8 (OCP e4m3) KV cache on gfx950: every kernel that writes or reads the
cache against the fp32 reference over the same e4m3 bytes
(``dmcp.ops.reference.kv_encode`` / ``kv_float``).

Writers: rope_kv, the fused QKV GEMM's RoPE/KV-append epilogue.  Readers:
the MFMA per-row decode kernel, the shared-prefix MFMA kernel, the prefill
kernel.  Plus the model end to end (fp8 vs bf16 cache)."""
import math
import os

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


def _f8(*shape, seed=0):
    from dmcp.ops.reference import kv_encode
    return kv_encode(_bf(*shape, seed=seed), torch.uint8)


def _close_fp8(got: torch.Tensor, exp: torch.Tensor):
    """Dequantised caches equal up to one e4m3 rounding step (the kernel
    rounds fp32 -> e4m3 once, the reference fp32 -> bf16 -> e4m3)."""
    from dmcp.ops.reference import kv_float
    a, b = kv_float(got), kv_float(exp)
    assert torch.isfinite(a).all()
    torch.testing.assert_close(a, b, atol=2 ** -9, rtol=0.13)
    assert (got == exp).float().mean().item() > 0.97


@pytest.mark.parametrize("D,Hq,Hkv", [(64, 32, 8), (128, 24, 8)])
def test_rope_kv_fp8(hip, D, Hq, Hkv):
    from dmcp.ops import reference
    T, S, MAXS = 13, 3, 64
    qkv = _bf(T, (Hq + 2 * Hkv) * D, seed=4, scale=3.0)
    qkv[0, (Hq + Hkv) * D] = 900.0  # a V value past the e4m3 range saturates
    pos = torch.arange(T, dtype=torch.int32, device="cuda") * 3 % MAXS
    slot = torch.arange(T, dtype=torch.int32, device="cuda") % S
    cs = reference.rope_tables(MAXS, D, device="cuda")
    kc = torch.zeros(S, Hkv, MAXS, D, dtype=torch.uint8, device="cuda")
    vc = torch.zeros_like(kc)
    kr, vr = kc.clone(), vc.clone()
    q = hip.rope_kv(qkv, pos, slot, cs, kc, vc, Hq)
    qr = reference.rope_kv(qkv, pos, slot, cs, kr, vr, Hq)
    torch.testing.assert_close(q.float(), qr.float(), atol=2e-2, rtol=1e-2)
    _close_fp8(kc, kr)
    assert torch.equal(vc, vr)  # bf16 -> e4m3 once on both sides
    assert reference.kv_float(vc[0, 0, 0, 0]).item() == 448.0


def test_fused_rope_kv_fp8(hip):
    """The fused QKV GEMM epilogue writes the same e4m3 cache as
    GEMM + rope_kv (bf16 q identical within the GEMM's rounding)."""
    from dmcp.ops import reference
    D, Hq, Hkv, K, M, S, MAXS = 64, 8, 2, 256, 5, 2, 32
    x = _bf(M, K, seed=1)
    w = _bf((Hq + 2 * Hkv) * D, K, seed=2, scale=0.05)
    pos = torch.arange(M, dtype=torch.int32, device="cuda") + 3
    slot = torch.tensor([0, 1, 0, 1, 0], dtype=torch.int32, device="cuda")
    cs = reference.rope_tables(MAXS, D, device="cuda")
    kc = torch.zeros(S, Hkv, MAXS, D, dtype=torch.uint8, device="cuda")
    vc = torch.zeros_like(kc)
    q = hip.fused_rope_kv(x, w, 1e-5, pos, slot, cs, kc, vc, Hq)
    h = reference.add_rmsnorm(x, torch.ones(K, dtype=torch.bfloat16, device="cuda"), 1e-5)
    qkv = (h.float() @ w.float().t()).to(torch.bfloat16)
    kr, vr = torch.zeros_like(kc), torch.zeros_like(vc)
    qr = reference.rope_kv(qkv, pos, slot, cs, kr, vr, Hq)
    torch.testing.assert_close(q.float(), qr.float(), atol=3e-2, rtol=3e-2)
    from dmcp.ops.reference import kv_float
    torch.testing.assert_close(kv_float(kc), kv_float(kr), atol=3e-2, rtol=0.13)
    torch.testing.assert_close(kv_float(vc), kv_float(vr), atol=3e-2, rtol=0.13)


@pytest.mark.parametrize("D,Hq,Hkv", [(64, 32, 8), (128, 24, 8)])
@pytest.mark.parametrize("P", [0, 45, 300])
def test_decode_attention_fp8(hip, D, Hq, Hkv, P):
    from dmcp.ops import reference
    from dmcp.ops.reference import SharedPrefix
    MAXS, S, B = 1024, 6, 9
    q = _bf(B, Hq, D, seed=11)
    kc = _f8(S + 1, Hkv, MAXS, D, seed=12)
    vc = _f8(S + 1, Hkv, MAXS, D, seed=13)
    pslot = S
    pre = None
    if P:
        pre = SharedPrefix(kc[pslot], vc[pslot], torch.tensor([P], dtype=torch.int32, device="cuda"))
    slot = torch.tensor([(b * 5) % S for b in range(B)], dtype=torch.int32, device="cuda")
    lens = torch.tensor([min(MAXS, P + 1 + (b * 97) % 700) for b in range(B)], dtype=torch.int32, device="cuda")
    scale = 1 / math.sqrt(D)
    for splits in (1, 4):
        got = hip.decode_attention(q, kc, vc, slot, lens, scale, prefix=pre, splits=splits)
        exp = reference.decode_attention(q, kc, vc, slot, lens, scale, prefix=pre)
        torch.testing.assert_close(got.float(), exp.float(), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("D,Hq,Hkv", [(64, 32, 8), (64, 16, 2), (128, 24, 8)])
@pytest.mark.parametrize("T,start,P", [(37, 0, 0), (129, 45, 45), (200, 700, 513)])
def test_prefill_attention_fp8(hip, D, Hq, Hkv, T, start, P):
    from dmcp.ops import reference
    MAXS, S = 1024, 4
    q = _bf(T, Hq, D, seed=T)
    kc = _f8(S, Hkv, MAXS, D, seed=T + 1)
    vc = _f8(S, Hkv, MAXS, D, seed=T + 2)
    kc[1, :, start + T:] = 0x7F  # e4m3 NaN where no query may look
    vc[1, :, start + T:] = 0x7F
    scale = 1 / math.sqrt(D)
    pslot = S - 1 if P else None
    exp = reference.prefill_attention(q, kc, vc, 1, start, pslot, P, scale)
    for variant in hip.PREFILL_VARIANTS[D]:
        got = hip.prefill_attention(q, kc, vc, 1, start, pslot, P, scale, variant=variant)
        assert torch.isfinite(got.float()).all()
        torch.testing.assert_close(got.float(), exp.float(), atol=2e-2, rtol=2e-2)


def test_model_fp8_kv_tracks_bf16():
    """dmcp-coder-1b heads, 2 layers: prefill after a shared prefix, then a
    batched decode step, fp8 cache vs bf16 cache (same weights)."""
    from dmcp.models.llm import LocalLM, preset
    cfg = preset("dmcp-coder-1b", layers=2, max_batch=4, max_seq=1024)
    a = LocalLM(cfg, device="cuda:0")
    b = LocalLM(preset("dmcp-coder-1b", layers=2, max_batch=4, max_seq=1024, kv_dtype="fp8"), device="cuda:0",
                weights=a.w)
    assert b.k_cache.dtype == torch.uint8
    g = torch.Generator().manual_seed(5)
    prefix = torch.randint(0, 256, (300,), generator=g).tolist()
    rest = torch.randint(0, 256, (120,), generator=g, dtype=torch.int32)
    outs = []
    for m in (a, b):
        P = m.set_prefix(prefix)
        for s in range(2):
            m.fork_prefix(s)
            m.forward_tokens(rest, s, P)
        toks = torch.tensor([65, 66], dtype=torch.int32, device="cuda")
        slots = torch.tensor([0, 1], dtype=torch.int32, device="cuda")
        pos = torch.full((2,), P + 120, dtype=torch.int32, device="cuda")
        outs.append(m.decode(toks, slots, pos).float())
        m.clear_prefix()
    cos = torch.nn.functional.cosine_similarity(outs[0], outs[1], dim=1)
    assert cos.min().item() > 0.99, cos
