"""MFMA prefill / extend attention (csrc/prefill_attn.hip) against the fp32
PyTorch reference (``dmcp.ops.reference.prefill_attention``).

Covers: plain causal prefill (start 0), extend after cached keys, the shared
prefix read in place from another slot, every GQA group size (1, 2, 3, 4,
8), both head dims, both unit counts per wave, partial query / key tiles,
stale NaN cache contents that must never be read, and a late-growing score
maximum (the online-softmax rescale path, rule 26 of the guide: bounded
random data alone rarely takes it)."""
import math

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


def _case(D, Hq, Hkv, T, start, P, MAXS=1024, S=4, seed=0):
    q = _bf(T, Hq, D, seed=seed + 1)
    kc = _bf(S, Hkv, MAXS, D, seed=seed + 2)
    vc = _bf(S, Hkv, MAXS, D, seed=seed + 3)
    slot, pslot = 1, S - 1
    nan = float("nan")
    # never-visible regions hold NaN: after the last query's position, and
    # (when the prefix is read in place) the slot's own copy of the prefix
    kc[slot, :, start + T:] = nan
    vc[slot, :, start + T:] = nan
    if P:
        kc[slot, :, :P] = nan
        vc[slot, :, :P] = nan
        kc[pslot, :, P:] = nan
        vc[pslot, :, P:] = nan
    return q, kc, vc, slot, pslot


@pytest.mark.parametrize("D,Hq,Hkv", [(64, 32, 8), (64, 8, 8), (64, 16, 8), (64, 24, 8), (64, 16, 2),
                                      (128, 24, 8), (128, 8, 4), (128, 16, 2)])
@pytest.mark.parametrize("T,start,P", [(1, 0, 0), (37, 0, 0), (300, 0, 0), (129, 45, 45), (200, 700, 513),
                                       (5, 256, 256), (64, 100, 0)])
def test_prefill_attention(hip, D, Hq, Hkv, T, start, P):
    from dmcp.ops import reference
    q, kc, vc, slot, pslot = _case(D, Hq, Hkv, T, start, P, seed=T + start)
    scale = 1 / math.sqrt(D)
    exp = reference.prefill_attention(q, kc.nan_to_num(), vc.nan_to_num(), slot, start,
                                      pslot if P else None, P, scale)
    for variant in hip.PREFILL_VARIANTS[D]:
        for nsplit in (1, 3):
            got = hip.prefill_attention(q, kc, vc, slot, start, pslot if P else None, P, scale, variant=variant,
                                        nsplit=nsplit)
            assert torch.isfinite(got.float()).all(), f"variant {variant} nsplit {nsplit}: non-finite output"
            torch.testing.assert_close(got.float(), exp.float(), atol=2e-2, rtol=2e-2)


def test_prefill_attention_growing_max(hip):
    """Scores grow along the key axis, so the running max moves on almost
    every tile and the O / l rescale runs with real weight behind it."""
    from dmcp.ops import reference
    D, Hq, Hkv, T, MAXS = 64, 32, 8, 160, 512
    q = _bf(T, Hq, D, seed=21).abs()
    kc = _bf(2, Hkv, MAXS, D, seed=22).abs()
    vc = _bf(2, Hkv, MAXS, D, seed=23)
    ramp = (torch.arange(MAXS, device="cuda", dtype=torch.float32) / 64.0 + 0.2)[None, None, :, None]
    kc = (kc.float() * ramp).to(torch.bfloat16)
    start = 90
    exp = reference.prefill_attention(q, kc, vc, 0, start, None, 0, 0.125)
    for variant in (0, 1):
        for nsplit in (1, 2, 5):
            got = hip.prefill_attention(q, kc, vc, 0, start, None, 0, 0.125, variant=variant, nsplit=nsplit)
            torch.testing.assert_close(got.float(), exp.float(), atol=3e-2, rtol=3e-2)


def test_prefill_attention_validates(hip):
    from dmcp.ops.hip import HipOpsError
    q = _bf(8, 8, 64)
    kc = _bf(2, 2, 64, 64)
    with pytest.raises(HipOpsError):
        hip.prefill_attention(q, kc, kc, 0, 60, None, 0, 0.1)  # past max_seq
    with pytest.raises(HipOpsError):
        hip.prefill_attention(q, kc, kc, 2, 0, None, 0, 0.1)  # bad slot
    with pytest.raises(HipOpsError):
        hip.prefill_attention(q, kc, kc, 0, 4, 1, 10, 0.1)  # prefix longer than start
    with pytest.raises(HipOpsError):
        hip.prefill_attention(q, kc, kc, 0, 0, None, 0, 0.1, out=torch.empty(3, device="cuda",
                                                                              dtype=torch.bfloat16))


def test_model_prefill_kernel_matches_sdpa_path():
    """forward_tokens with the MFMA kernel (prefix read in place) == the SDPA
    path (prefix copied into the slot) on the 1B geometry's head layout."""
    from dmcp.models.llm import LocalLM, preset
    cfg = preset("tiny", max_batch=4, max_seq=512, n_heads=8, n_kv_heads=2, head_dim=64, layers=2)
    a = LocalLM(cfg, device="cuda:0")
    b = LocalLM(cfg, device="cuda:0", weights=a.w)
    assert a.use_prefill_kernel
    b.use_prefill_kernel = False
    g = torch.Generator().manual_seed(3)
    prefix = torch.randint(0, 256, (150,), generator=g).tolist()
    rest = torch.randint(0, 256, (97,), generator=g, dtype=torch.int32)
    outs = []
    for m in (a, b):
        P = m.set_prefix(prefix)
        start = m.fork_prefix(2)
        assert start == P == 150
        outs.append(m.forward_tokens(rest, 2, start).float())
        m.clear_prefix()
    torch.testing.assert_close(outs[0], outs[1], atol=5e-2, rtol=5e-2)
    assert a._slot_prefix == {}


@pytest.mark.parametrize("D,Hq,Hkv", [(64, 32, 8), (64, 16, 2), (128, 24, 8)])
@pytest.mark.parametrize("kv", ["bf16", "fp8"])
def test_prefill_varlen_matches_per_sequence_reference(hip, D, Hq, Hkv, kv):
    """One packed launch over sequences of mixed lengths (1 token to a few
    hundred, partial tiles), some after the shared prefix read in place from
    the prefix slot, some plain prefills, one extending its own cached keys
    == the fp32 reference of each sequence; stale NaN cache regions past each
    sequence's end (and the prefix range of the own slot) are never read."""
    from dmcp.ops import reference
    MAXS, S = 1024, 8
    pslot, P = S - 1, 300
    scale = 1 / math.sqrt(D)
    seqs = [(1, P, P), (157, P, P), (33, 0, 0), (260, P, P), (5, 0, 0), (96, 512, 0)]  # (T, start, prefix len)
    Ttot = sum(t for t, _, _ in seqs)
    q = _bf(Ttot, Hq, D, seed=5)
    kc = _bf(S, Hkv, MAXS, D, seed=6)
    vc = _bf(S, Hkv, MAXS, D, seed=7)
    if kv == "fp8":
        kc, vc = reference.kv_encode(kc.float(), torch.uint8), reference.kv_encode(vc.float(), torch.uint8)
    nanv = 0x7F if kv == "fp8" else float("nan")  # e4m3 0x7f is NaN
    offsets, slots, starts, plens = [0], [], [], []
    for i, (T, st, pl) in enumerate(seqs):
        slots.append(i)
        starts.append(st)
        plens.append(pl)
        offsets.append(offsets[-1] + T)
    ref_k, ref_v = kc.clone(), vc.clone()
    for i, (T, st, pl) in enumerate(seqs):
        kc[i, :, st + T:] = nanv
        vc[i, :, st + T:] = nanv
        if pl:
            kc[i, :, :pl] = nanv
            vc[i, :, :pl] = nanv
    kc[pslot, :, P:] = nanv
    vc[pslot, :, P:] = nanv
    exp = reference.prefill_attention_varlen(q, ref_k, ref_v, offsets, slots, starts, pslot, plens, scale)
    got = hip.prefill_attention_varlen(q, kc, vc, offsets, slots, starts, pslot, plens, scale)
    assert torch.isfinite(got.float()).all()
    torch.testing.assert_close(got.float(), exp.float(), atol=3e-2, rtol=3e-2)
    # single sequences through the varlen launch == the single-sequence kernel
    one = hip.prefill_attention_varlen(q[:157 + 1][1:], kc, vc, [0, 157], [1], [P], pslot, [P], scale)
    solo = hip.prefill_attention(q[1:158], kc, vc, 1, P, pslot, P, scale, nsplit=1)
    torch.testing.assert_close(one.float(), solo.float(), atol=1e-2, rtol=1e-2)


def test_prefill_varlen_rejects_bad_tables(hip):
    q = _bf(10, 8, 64)
    kc = _bf(2, 2, 64, 64)
    with pytest.raises(hip.HipOpsError):  # past the cache capacity
        hip.prefill_attention_varlen(q, kc, kc, [0, 10], [0], [60])
    with pytest.raises(hip.HipOpsError):  # offsets do not cover q
        hip.prefill_attention_varlen(q, kc, kc, [0, 9], [0], [0])
    with pytest.raises(hip.HipOpsError):  # prefix longer than the start
        hip.prefill_attention_varlen(q, kc, kc, [0, 10], [0], [3], 1, [5])


@pytest.mark.parametrize("kv", ["bf16", "fp8"])
def test_model_prefill_batch_matches_reference(kv):
    """LocalLM.prefill_batch (packed GEMMs + varlen attention) == one
    forward_tokens per sequence and the fp32 reference model, with and without
    the shared prefix."""
    from dmcp.models.llm import LocalLM, preset
    m = LocalLM(preset("tiny", max_batch=8, kv_dtype=kv), device="cuda", seed=9)
    seqs = [[256] + list(b"class A { void a() {} }"), [256] + list(b"interface Bee { int b(); long c(); }"),
            [256, 65]]
    single = [m.forward_tokens(torch.tensor(t, dtype=torch.int32), s, 0).float() for s, t in enumerate(seqs)]
    got = m.prefill_batch([(t, s + 3, 0) for s, t in enumerate(seqs)]).float()
    for g, one, t in zip(got, single, seqs):
        ref = m.reference_logits(t)[-1].float()
        assert (g - ref).abs().max().item() / max(1.0, ref.abs().max().item()) < 0.05
        assert (g - one).abs().max().item() / max(1.0, one.abs().max().item()) < 0.03
    prefix = [256] + list(b"Shared instructions and the README of the project. " * 3)
    P = m.set_prefix(prefix)
    try:
        for s in range(len(seqs)):
            m.fork_prefix(s)
        got = m.prefill_batch([(t[1:], s, P) for s, t in enumerate(seqs)]).float()
        for g, t in zip(got, seqs):
            ref = m.reference_logits(prefix + t[1:])[-1].float()
            assert (g - ref).abs().max().item() / max(1.0, ref.abs().max().item()) < 0.05
    finally:
        m.clear_prefix()
