"""Numerics of the gfx950 HIP kernels against plain PyTorch fp32 references."""
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


@pytest.mark.parametrize("H", [256, 2048, 3072, 8192])
@pytest.mark.parametrize("with_res", [False, True])
def test_add_rmsnorm(hip, H, with_res):
    from dmcp.ops import reference
    x = _bf(37, H, seed=1)
    w = _bf(H, seed=2)
    res = _bf(37, H, seed=3) if with_res else None
    res_ref = res.clone() if with_res else None
    got = hip.add_rmsnorm(x, w, 1e-5, residual=res)
    exp = reference.add_rmsnorm(x.float().to(torch.bfloat16), w, 1e-5, residual=res_ref)
    torch.testing.assert_close(got.float(), exp.float(), atol=3e-2, rtol=2e-2)
    if with_res:
        assert torch.equal(res, res_ref)


@pytest.mark.parametrize("D,Hq,Hkv", [(64, 32, 8), (128, 24, 8), (64, 4, 4)])
def test_rope_kv(hip, D, Hq, Hkv):
    from dmcp.ops import reference
    T, S, MAXS = 13, 3, 64
    qkv = _bf(T, (Hq + 2 * Hkv) * D, seed=4)
    pos = torch.randint(0, MAXS, (T,), dtype=torch.int32, device="cuda")
    slot = torch.randint(0, S, (T,), dtype=torch.int32, device="cuda")
    # make (slot, pos) unique so the reference's sequential writes equal the kernel's
    pos = torch.arange(T, dtype=torch.int32, device="cuda") * 3 % MAXS
    cs = reference.rope_tables(MAXS, D, device="cuda")
    kc = torch.zeros(S, Hkv, MAXS, D, dtype=torch.bfloat16, device="cuda")
    vc = torch.zeros_like(kc)
    kr, vr = kc.clone(), vc.clone()
    q = hip.rope_kv(qkv, pos, slot, cs, kc, vc, Hq)
    qr = reference.rope_kv(qkv, pos, slot, cs, kr, vr, Hq)
    torch.testing.assert_close(q.float(), qr.float(), atol=2e-2, rtol=1e-2)
    torch.testing.assert_close(kc.float(), kr.float(), atol=2e-2, rtol=1e-2)
    assert torch.equal(vc, vr)


def test_rope_kv_skips_invalid_slot(hip):
    from dmcp.ops import reference
    D, Hq, Hkv, S, MAXS = 64, 4, 2, 2, 16
    qkv = _bf(2, (Hq + 2 * Hkv) * D)
    cs = reference.rope_tables(MAXS, D, device="cuda")
    kc = torch.zeros(S, Hkv, MAXS, D, dtype=torch.bfloat16, device="cuda")
    vc = torch.zeros_like(kc)
    hip.rope_kv(qkv, torch.tensor([0, 99], dtype=torch.int32, device="cuda"),
                torch.tensor([-1, 0], dtype=torch.int32, device="cuda"), cs, kc, vc, Hq)
    assert kc.abs().sum().item() == 0 and vc.abs().sum().item() == 0


@pytest.mark.parametrize("D,Hq,Hkv,MAXS", [(64, 32, 8, 1024), (128, 16, 4, 300), (64, 8, 8, 64), (128, 8, 1, 2048),
                                           (128, 24, 8, 700), (64, 12, 2, 513)])
def test_decode_attention(hip, D, Hq, Hkv, MAXS):
    from dmcp.ops import reference
    B, S = 5, 7
    q = _bf(B, Hq, D, seed=5)
    kc = _bf(S, Hkv, MAXS, D, seed=6)
    vc = _bf(S, Hkv, MAXS, D, seed=7)
    slot = torch.tensor([3, 0, 6, 1, 5], dtype=torch.int32, device="cuda")
    lens = torch.tensor([1, MAXS, max(1, MAXS // 3), 17 % MAXS + 1, MAXS - 1], dtype=torch.int32, device="cuda")
    scale = 1 / math.sqrt(D)
    got = hip.decode_attention(q, kc, vc, slot, lens, scale)
    exp = reference.decode_attention(q, kc, vc, slot, lens, scale)
    torch.testing.assert_close(got.float(), exp.float(), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("D,Hq,Hkv", [(64, 32, 8), (64, 8, 4), (128, 24, 8), (64, 16, 2)])
@pytest.mark.parametrize("P", [1, 45, 256, 700])
@pytest.mark.parametrize("B", [1, 9, 70])
def test_decode_attention_shared_prefix(hip, D, Hq, Hkv, P, B):
    """MFMA shared-prefix kernel + per-row suffix + merge == fp32 attention
    over [prefix ++ own keys]; odd P / B exercise partial key and query tiles."""
    from dmcp.ops import reference
    from dmcp.ops.reference import SharedPrefix
    MAXS, S = 1024, 6
    q = _bf(B, Hq, D, seed=11)
    kc = _bf(S + 1, Hkv, MAXS, D, seed=12)
    vc = _bf(S + 1, Hkv, MAXS, D, seed=13)
    pslot = S  # the prefix lives in the last slot
    plen = torch.tensor([P], dtype=torch.int32, device="cuda")
    slot = torch.tensor([(b * 5) % S for b in range(B)], dtype=torch.int32, device="cuda")
    slot[B // 2] = -1  # a padding row
    lens = torch.tensor([min(MAXS, P + 1 + (b * 37) % 300) for b in range(B)], dtype=torch.int32, device="cuda")
    scale = 1 / math.sqrt(D)
    pre = SharedPrefix(kc[pslot], vc[pslot], plen)
    exp = reference.decode_attention(q, kc, vc, slot, lens, scale, prefix=pre)
    for chunk in (256, 1024):
        for sp in ("1", "5", "16"):  # prefix key splits (DMCP_PREFIX_SPLITS)
            os.environ["DMCP_PREFIX_SPLITS"] = sp
            try:
                got = hip.decode_attention(q, kc, vc, slot, lens, scale, chunk=chunk, prefix=pre)
            finally:
                os.environ.pop("DMCP_PREFIX_SPLITS")
            torch.testing.assert_close(got.float(), exp.float(), atol=2e-2, rtol=2e-2)
            assert got[B // 2].abs().sum().item() == 0
    # a workspace too small for the prefix partials is refused (never overrun)
    ws = hip.decode_workspace(B, Hq, Hkv, D, 256, "cuda", chunk=256, prefix_slots=0)
    with pytest.raises(hip.HipOpsError):
        hip.decode_attention(q, kc, vc, slot, lens, scale, workspace=ws, chunk=256, prefix=pre, splits=1)
    # length 0 in device memory: the prefix kernel is a no-op, rows read their own keys
    plen.zero_()
    got = hip.decode_attention(q, kc, vc, slot, lens, scale, prefix=pre)
    exp = reference.decode_attention(q, kc, vc, slot, lens, scale)
    torch.testing.assert_close(got.float(), exp.float(), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("splits", [1, 3, 6])
@pytest.mark.parametrize("P", [0, 300])
def test_decode_attention_balanced_splits(hip, splits, P):
    """Equal per-row splits (decode_plan: at most ``splits`` parts of >= chunk
    keys, rounded to 32-key tiles), with and without a shared prefix;
    lengths hit partial tiles and split boundaries.  With one split per row
    the main kernel merges the prefix partials itself (no combine pass),
    including a row that has no keys of its own."""
    from dmcp.ops import reference
    from dmcp.ops.reference import SharedPrefix
    D, Hq, Hkv, MAXS, S = 64, 32, 8, 1024, 9
    lens_own = [1, 31, 32, 33, 257, 700, 1000 - P, 2, 511] + ([0] if P else [])  # 0: prefix keys only
    B = len(lens_own)
    q = _bf(B, Hq, D, seed=21)
    kc = _bf(S + 1, Hkv, MAXS, D, seed=22)
    vc = _bf(S + 1, Hkv, MAXS, D, seed=23)
    slot = torch.tensor([(3 * b) % S for b in range(B)], dtype=torch.int32, device="cuda")
    lens = torch.tensor([P + n for n in lens_own], dtype=torch.int32, device="cuda")
    pre = None
    if P:
        pre = SharedPrefix(kc[S], vc[S], torch.tensor([P], dtype=torch.int32, device="cuda"))
    got = hip.decode_attention(q, kc, vc, slot, lens, 0.125, chunk=64, prefix=pre, splits=splits)
    exp = reference.decode_attention(q, kc, vc, slot, lens, 0.125, prefix=pre)
    torch.testing.assert_close(got.float(), exp.float(), atol=2e-2, rtol=2e-2)


def test_decode_plan_targets_busy_waves(hip):
    chunk, splits = hip.decode_plan(96, 8, 8192)
    assert chunk == 256 and 96 * 8 * splits >= 4096 and splits <= 32
    assert hip.decode_plan(1, 8, 1024) == (256, 4)  # capped by max_seq / chunk
    with pytest.raises(hip.HipOpsError):
        hip.decode_attention(_bf(1, 8, 64), _bf(1, 2, 64, 64), _bf(1, 2, 64, 64),
                             torch.zeros(1, dtype=torch.int32, device="cuda"),
                             torch.ones(1, dtype=torch.int32, device="cuda"), 0.1, chunk=32, splits=3)


def test_decode_attention_bad_slot_is_zero(hip):
    D, Hq, Hkv, MAXS = 64, 8, 2, 128
    q = _bf(2, Hq, D)
    kc = _bf(2, Hkv, MAXS, D)
    got = hip.decode_attention(q, kc, kc.clone(), torch.tensor([-1, 5], dtype=torch.int32, device="cuda"),
                               torch.tensor([10, 10], dtype=torch.int32, device="cuda"), 0.125)
    assert got.abs().sum().item() == 0


@pytest.mark.parametrize("T,I", [(1, 8192), (33, 512), (7, 1000)])
def test_silu_mul(hip, T, I):
    from dmcp.ops import reference
    gu = _bf(T, 2 * I, seed=8, scale=3)
    torch.testing.assert_close(hip.silu_mul(gu).float(), reference.silu_mul(gu).float(), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("V", [320, 32000])
def test_masked_argmax(hip, V):
    from dmcp.ops import reference
    from dmcp.enrich.local import _json_safe_mask
    B = 9
    logits = _bf(B, V, seed=9)
    assert torch.equal(hip.masked_argmax(logits), reference.masked_argmax(logits))
    mask = torch.tensor([_json_safe_mask(V, b % 2 == 0) for b in range(B)], dtype=torch.int32, device="cuda")
    got = hip.masked_argmax(logits, mask, vocab=V)
    exp = reference.masked_argmax(logits, mask, vocab=V)
    assert torch.equal(got, exp)
    assert all(0x20 <= int(t) < 0x7F for t in got)


@pytest.mark.parametrize("B,ld,V", [(64, 128256, 128256), (5, 1003, 1003), (7, 1008, 1003), (3, 40, 17)])
def test_masked_argmax_chunks_tail_ties(hip, B, ld, V):
    """The 16-B chunk path (ld % 8 == 0), the element-wise path (ld % 8 != 0)
    and the ids past the last whole chunk, against the fp32 reference, with
    a mask table + mask_idx, ties (lowest id wins) and a row with nothing
    allowed (id 0)."""
    from dmcp.ops import reference
    g = torch.Generator().manual_seed(B * 7 + V)
    # few distinct values: many exact ties
    logits = (torch.randint(0, 5, (B, ld), generator=g).float() / 4).to(torch.bfloat16).cuda()
    W = (V + 31) // 32
    bits = torch.randint(0, 2, (4, V), generator=g, dtype=torch.int64)
    bits[1] = 0  # nothing allowed
    bits[2] = 1
    words = torch.zeros(4, W, dtype=torch.int64)
    for j in range(32):
        col = bits[:, j::32]
        words[:, :col.shape[1]] |= col << j
    mask = ((words + 2 ** 31) % 2 ** 32 - 2 ** 31).to(torch.int32).cuda()  # uint32 bit patterns
    midx = torch.randint(-1, 6, (B,), generator=g, dtype=torch.int32).cuda()  # clamped to [0, 4)
    got = hip.masked_argmax(logits, mask, vocab=V, mask_idx=midx)
    exp = reference.masked_argmax(logits, mask, vocab=V, mask_idx=midx)
    assert torch.equal(got.cpu(), exp.cpu())
    assert torch.equal(hip.masked_argmax(logits, vocab=V).cpu(), reference.masked_argmax(logits, vocab=V).cpu())
    if B >= 3:
        rows = midx.clamp(0, 3).cpu()
        assert all(int(got[i]) == 0 for i in range(B) if int(rows[i]) == 1)


def test_embedding(hip):
    from dmcp.ops import reference
    table = _bf(320, 2048, seed=10)
    ids = torch.tensor([0, 5, 319, 7, 7], dtype=torch.int32, device="cuda")
    assert torch.equal(hip.embedding(table, ids), reference.embedding(table, ids))


def test_shape_validation_raises(hip):
    with pytest.raises(hip.HipOpsError):
        hip.add_rmsnorm(_bf(2, 100), _bf(100), 1e-5)
    with pytest.raises(hip.HipOpsError):
        hip.decode_attention(_bf(1, 6, 64), _bf(1, 4, 8, 64), _bf(1, 4, 8, 64),
                             torch.zeros(1, dtype=torch.int32, device="cuda"),
                             torch.ones(1, dtype=torch.int32, device="cuda"), 0.1)
    # undersized caller-supplied output buffers are refused before the launch
    with pytest.raises(hip.HipOpsError):
        hip.add_rmsnorm(_bf(4, 128), _bf(128), 1e-5, out=_bf(3, 128))
    with pytest.raises(hip.HipOpsError):
        hip.silu_mul(_bf(4, 256), out=_bf(4, 64))
    with pytest.raises(hip.HipOpsError):
        hip.embedding(_bf(16, 64), torch.zeros(8, dtype=torch.int32, device="cuda"), out=_bf(7, 64))
    with pytest.raises(hip.HipOpsError):
        hip.masked_argmax(_bf(4, 64), out=torch.zeros(3, dtype=torch.int32, device="cuda"))
    with pytest.raises(hip.HipOpsError):
        hip.decode_attention(_bf(2, 4, 64), _bf(2, 4, 8, 64), _bf(2, 4, 8, 64),
                             torch.zeros(2, dtype=torch.int32, device="cuda"),
                             torch.ones(2, dtype=torch.int32, device="cuda"), 0.1, out=_bf(1, 4, 64))
    cos_sin = torch.zeros(16, 32, 2, dtype=torch.float32, device="cuda")
    with pytest.raises(hip.HipOpsError):
        hip.rope_kv(_bf(2, 6 * 64), torch.zeros(2, dtype=torch.int32, device="cuda"),
                    torch.zeros(2, dtype=torch.int32, device="cuda"), cos_sin, _bf(1, 1, 16, 64), _bf(1, 1, 16, 64),
                    4, q_out=_bf(1, 4, 64))


@pytest.mark.parametrize("H,with_norm,with_src", [(2048, True, True), (256, True, False), (4096, False, True),
                                                  (3072, True, True)])
def test_decode_embed_norm_matches_reference(H, with_norm, with_src):
    """Decode-step inputs in one launch (token select from the previous step's
    ids, embedding, first RMSNorm, seq_len) vs the fp32 reference."""
    from dmcp.ops import hip, reference
    g = torch.Generator().manual_seed(H)
    V, B = 320, 77
    table = torch.randn(V, H, generator=g).to(torch.bfloat16).cuda()
    w = (torch.rand(H, generator=g) + 0.5).to(torch.bfloat16).cuda() if with_norm else None
    tokens = torch.randint(-3, V + 3, (B,), generator=g, dtype=torch.int32).cuda()  # clamped like the embedding
    pos = torch.randint(0, 8000, (B,), generator=g, dtype=torch.int32).cuda()
    src = last = None
    if with_src:
        src = torch.randint(-1, 96, (B,), generator=g, dtype=torch.int32).cuda()
        last = torch.randint(0, V, (96,), generator=g, dtype=torch.int32).cuda()
    r, h, sl = hip.decode_embed_norm(table, tokens, pos, w, 1e-5, src, last)
    rr, hr, slr = reference.decode_embed_norm(table.cpu().float(), tokens.cpu(), pos.cpu(),
                                              None if w is None else w.cpu().float(), 1e-5,
                                              None if src is None else src.cpu(), None if last is None else last.cpu())
    assert torch.equal(r.cpu().float(), rr.float()) and torch.equal(sl.cpu(), slr)
    if with_norm:
        torch.testing.assert_close(h.cpu().float(), hr.float(), atol=2e-2, rtol=2e-2)
    else:
        assert h is None


@pytest.mark.parametrize("splits", [1, 4])
@pytest.mark.parametrize("B", [3, 40, 97])
def test_decode_attention_rows_off_the_prefix(hip, splits, B):
    """Rows flagged 0 in prefix.rows (another project's sequences, admitted
    while this prefix is resident) attend to their own slot from key 0; the
    flagged rows keep the shared prefix -- both in one launch, vs fp32."""
    from dmcp.ops import reference
    from dmcp.ops.reference import SharedPrefix
    D, Hq, Hkv, MAXS, S, P = 64, 32, 8, 1024, 8, 333
    q = _bf(B, Hq, D, seed=31)
    kc = _bf(S + 1, Hkv, MAXS, D, seed=32)
    vc = _bf(S + 1, Hkv, MAXS, D, seed=33)
    slot = torch.tensor([b % S for b in range(B)], dtype=torch.int32, device="cuda")
    rows = torch.tensor([b % 3 != 1 for b in range(B)], dtype=torch.int32, device="cuda")
    lens = torch.tensor([P + 1 + (b * 53) % 600 for b in range(B)], dtype=torch.int32, device="cuda")
    pre = SharedPrefix(kc[S], vc[S], torch.tensor([P], dtype=torch.int32, device="cuda"), rows)
    got = hip.decode_attention(q, kc, vc, slot, lens, 0.125, chunk=64, prefix=pre, splits=splits)
    exp = reference.decode_attention(q, kc, vc, slot, lens, 0.125, prefix=pre)
    torch.testing.assert_close(got.float(), exp.float(), atol=2e-2, rtol=2e-2)
    # unflagged rows == no prefix at all
    off = rows.cpu() == 0
    plain = reference.decode_attention(q, kc, vc, slot, lens, 0.125)
    torch.testing.assert_close(got[off.cuda()].float(), plain[off].float(), atol=2e-2, rtol=2e-2)


def test_decode_embed_norm_switches_the_grammar_mask(hip):
    """A gathered token equal to alt_token switches that row's mask index to
    mask_alt (where >= 0); literal rows and other tokens keep theirs."""
    from dmcp.ops import reference
    g = torch.Generator().manual_seed(5)
    V, H, B, Q = 320, 256, 64, 34
    table = torch.randn(V, H, generator=g).to(torch.bfloat16).cuda()
    tokens = torch.randint(0, V, (B,), generator=g, dtype=torch.int32)
    pos = torch.arange(B, dtype=torch.int32)
    src = torch.tensor([b % 4 - 1 for b in range(B)], dtype=torch.int32)  # -1 literal, else gathered
    last = torch.tensor([Q, 7, Q], dtype=torch.int32)
    midx = torch.tensor([b % 2 for b in range(B)], dtype=torch.int32)
    alt = torch.tensor([5 if b % 5 else -1 for b in range(B)], dtype=torch.int32)
    m_hip = midx.clone().cuda()
    hip.decode_embed_norm(table, tokens.cuda(), pos.cuda(), None, 1e-5, src.cuda(), last.cuda(), m_hip, alt.cuda(), Q)
    m_ref = midx.clone()
    reference.decode_embed_norm(table.cpu().float(), tokens, pos, None, 1e-5, src, last, m_ref, alt, Q)
    assert torch.equal(m_hip.cpu(), m_ref)
    exp = [5 if (s >= 0 and int(last[s]) == Q and a >= 0) else int(m) for s, a, m in zip(src, alt, midx)]
    assert m_ref.tolist() == exp and exp != midx.tolist()


@pytest.mark.parametrize("kv", ["bf16", "fp8"])
def test_kv_fork_matches_indexed_copy(kv):
    """hip.kv_fork (one launch, both caches, every layer) writes exactly what
    the indexed copy cache[:, dsts, :, a:b] = cache[:, src, :, a:b] does, and
    nothing outside [a, b) or the destination slots."""
    from dmcp.ops import hip
    dt = torch.uint8 if kv == "fp8" else torch.bfloat16
    g = torch.Generator(device="cuda").manual_seed(3)
    shape = (3, 40, 8, 256, 64)
    if dt == torch.uint8:
        kc = torch.randint(0, 120, shape, generator=g, device="cuda", dtype=torch.uint8)
    else:
        kc = torch.randn(shape, generator=g, device="cuda").to(dt)
    vc = kc.flip(0).contiguous()
    for src, dsts, a, b in ((5, [7, 0, 39], 17, 200), (2, list(range(8, 44 - 4)), 0, 256), (1, [3], 255, 256)):
        rk, rv = kc.clone(), vc.clone()
        idx = torch.tensor(dsts, device="cuda")
        for r in (rk, rv):
            r[:, idx, :, a:b] = r[:, src, :, a:b].unsqueeze(1)
        hip.kv_fork(kc, vc, src, dsts, a, b)
        torch.cuda.synchronize()
        assert torch.equal(kc, rk) and torch.equal(vc, rv)


@pytest.mark.parametrize("kv", ["bf16", "fp8"])
@pytest.mark.parametrize("splits", [1, 4])
@pytest.mark.parametrize("P", [0, 300])
def test_decode_attention_fork_table(hip, kv, splits, P):
    """Method branches (fork table: slot -> (parent slot, end)): a row reads
    its keys below ``end`` from the parent slot in place.  Bit-identical to
    the same kernel on caches where those keys were copied into the row's
    slot; fork ends inside a 32-key tile, on a tile edge, past the row's
    length; a shared prefix in front; rows without a parent unchanged.  Also
    within bf16 tolerance of reference.decode_attention(..., fork=) in fp32."""
    from dmcp.ops.reference import SharedPrefix
    D, Hq, Hkv, MAXS, S = 64, 32, 8, 1024, 10
    dt = torch.uint8 if kv == "fp8" else torch.bfloat16

    def cache(seed):
        x = _bf(S + 1, Hkv, MAXS, D, seed=seed)
        return x.to(torch.float8_e4m3fn).view(torch.uint8) if kv == "fp8" else x
    kc, vc = cache(31), cache(32)
    rows = [(1, None, 700), (2, (1, P + 77), 690), (3, (1, P + 96), 500), (4, (1, P + 600), 420),
            (5, None, P + 3), (6, (5, P + 2), P + 40)]
    B = len(rows)
    q = _bf(B, Hq, D, seed=33)
    slot = torch.tensor([r[0] for r in rows], dtype=torch.int32, device="cuda")
    lens = torch.tensor([max(r[2], P + 1) for r in rows], dtype=torch.int32, device="cuda")
    fork = torch.stack([torch.arange(S + 1), torch.zeros(S + 1, dtype=torch.long)], 1).to(torch.int32).cuda()
    kc2, vc2 = kc.clone(), vc.clone()
    for b, (s, par, _) in enumerate(rows):
        if par is not None:
            fork[s] = torch.tensor(par, dtype=torch.int32)
            e = min(par[1], int(lens[b]))
            kc2[s, :, P:e], vc2[s, :, P:e] = kc[par[0], :, P:e], vc[par[0], :, P:e]
    pre = pre2 = None
    if P:
        pl = torch.tensor([P], dtype=torch.int32, device="cuda")
        pre, pre2 = SharedPrefix(kc[S], vc[S], pl), SharedPrefix(kc2[S], vc2[S], pl)
    got = hip.decode_attention(q, kc, vc, slot, lens, 0.125, chunk=64, prefix=pre, splits=splits, fork=fork)
    exp = hip.decode_attention(q, kc2, vc2, slot, lens, 0.125, chunk=64, prefix=pre2, splits=splits)
    assert torch.equal(got, exp)
    assert dt == kc.dtype
    # and against the fp32 reference reading the parents' keys through the same fork table
    from dmcp.ops import reference
    ref = reference.decode_attention(q, kc, vc, slot, lens, 0.125, prefix=pre, fork=fork)
    torch.testing.assert_close(got.float(), ref.float(), atol=2e-2, rtol=2e-2)

