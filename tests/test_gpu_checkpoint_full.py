"""A full-size Llama-format checkpoint through ``load_safetensors`` on the
GPU (round-6 verdict item 9): Llama-3.2-1B geometry -- 16 layers, hidden
2,048, 32 / 8 heads of 64, intermediate 8,192, a 128,256-id vocabulary --
with *trained-like* weights: heavy-tailed matrices (a Gaussian scale
mixture), non-trivial RMSNorm weights, and a few residual channels carried
at ~100x the others (the outlier features of trained Llama checkpoints,
damped by small norm weights on those channels).  Written by the test (no
download); 2.5 GB of safetensors.

Checked against the fp32 reference model (``LocalLM.reference_logits``):

* the engine's batched prefill (its default GEMMs for a loaded checkpoint)
  -- last-position logit cosine >= 0.999, per-layer K/V of the prompt within
  4 % (relative Frobenius) of the fp32 K/V;
* a 768-row decode step on the default kernels (the large-tile trunk: its
  split-K GEMMs with the fused RoPE / KV-append and residual / RMSNorm
  reductions, the fused LM head + masked argmax): cosine >= 0.999 on the
  reference rows with a bf16 KV cache, >= 0.99 with the default fp8 one,
  argmax agreement of the fused head;
* the MXFP8 prefill (``prefill_dtype="fp8"``) on the same weights: logit
  cosine and top-1 agreement against fp32 -- the gate for using it on
  checkpoints (docs/PARITY.md)."""
import json
import os

import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

H, L, NH, NKV, D, INTER, V = 2048, 16, 32, 8, 64, 8192, 128256
OUTLIERS = (7, 300, 1029, 1800)  # residual channels at ~100x


@pytest.fixture(scope="module")
def ckpt(tmp_path_factory):
    from dmcp.utils import synth
    return synth.llama_checkpoint(str(tmp_path_factory.mktemp("ckpt_full")), outliers=OUTLIERS)


def _load(ckpt, **kw):
    from dmcp.models.llm import LocalLM
    from dmcp.ops import hip
    hip.lib()
    return LocalLM.load_safetensors(ckpt, device="cuda", **kw)


def _prompts(n, gen):
    return [[128000] + torch.randint(0, V - 256, (int(l),), generator=gen).tolist()
            for l in torch.randint(40, 160, (n,), generator=gen)]


def _cos(a, b):
    return torch.nn.functional.cosine_similarity(a.float().flatten(), b.float().flatten(), dim=0).item()


def _ref_kv(model, toks):
    """fp32 K / V of every layer for a prompt (the reference model's own
    projections, RoPE on K)."""
    from dmcp import ops
    c = model.cfg
    w = {k: v.float() for k, v in model.w.items()}
    ids = torch.tensor(toks, device="cuda")
    T = ids.numel()
    x = w["embed"][ids]

    def rms(t, g):
        return t * torch.rsqrt(t.pow(2).mean(-1, keepdim=True) + c.eps) * g
    pos = torch.arange(T, device="cuda", dtype=torch.int32)
    G = c.n_heads // c.n_kv_heads
    ks, vs = [], []
    for i in range(c.layers):
        qkv = (rms(x, w[f"l{i}.ln1"]) @ w[f"l{i}.wqkv"].t()).view(T, c.n_heads + 2 * c.n_kv_heads, c.head_dim)
        q = ops.reference.apply_rope(qkv[:, :c.n_heads], pos, model.cos_sin)
        k = ops.reference.apply_rope(qkv[:, c.n_heads:c.n_heads + c.n_kv_heads], pos, model.cos_sin)
        v = qkv[:, c.n_heads + c.n_kv_heads:]
        ks.append(k)
        vs.append(v)
        kk, vv = k.repeat_interleave(G, 1), v.repeat_interleave(G, 1)
        att = torch.einsum("thd,shd->hts", q, kk) * model.scale
        att = att.masked_fill(torch.triu(torch.ones(T, T, dtype=torch.bool, device="cuda"), 1), float("-inf"))
        o = torch.einsum("hts,shd->thd", torch.softmax(att, -1), vv).reshape(T, -1)
        x = x + o @ w[f"l{i}.wo"].t()
        h = rms(x, w[f"l{i}.ln2"])
        gu = h @ w[f"l{i}.wgu"].t()
        x = x + (torch.nn.functional.silu(gu[:, :c.intermediate]) * gu[:, c.intermediate:]) @ w[f"l{i}.wdown"].t()
    return ks, vs


def test_full_checkpoint_prefill_and_kv_match_fp32(ckpt):
    from dmcp.ops.reference import kv_float
    m = _load(ckpt, max_batch=16, max_rows=1024, max_seq=1024, kv_dtype="bf16")
    assert m.checkpoint == ckpt and m.cfg.vocab_size == V and m.cfg.layers == L
    g = torch.Generator().manual_seed(1)
    prompts = _prompts(6, g)
    got = m.prefill_batch([(p, s, 0) for s, p in enumerate(prompts)]).float()
    coss, agree = [], []
    for s, p in enumerate(prompts):
        ref = m.reference_logits(p)[-1].float()
        coss.append(_cos(got[s], ref))
        agree.append(int(got[s].argmax()) == int(ref.argmax()))
    print("prefill logit cosine", [round(c, 5) for c in coss], "top-1", sum(agree), "/", len(agree))
    assert min(coss) >= 0.999, coss
    assert sum(agree) >= len(agree) - 1
    # per-layer K / V of the first prompt vs fp32: relative Frobenius error
    ks, vs = _ref_kv(m, prompts[0])
    T = len(prompts[0])
    errs = []
    for i in range(L):
        kg = kv_float(m.k_cache[i, 0, :, :T]).float().transpose(0, 1)  # [T, Hkv, D]
        vg = kv_float(m.v_cache[i, 0, :, :T]).float().transpose(0, 1)
        ek = ((kg - ks[i]).norm() / ks[i].norm()).item()
        ev = ((vg - vs[i]).norm() / vs[i].norm()).item()
        errs.append((round(ek, 4), round(ev, 4)))
    print("per-layer K/V relative error", errs)
    assert max(max(e) for e in errs) < 0.04, errs  # bf16 rounding compounding over 16 layers


@pytest.mark.parametrize("kv,bound", [("bf16", 0.999), ("fp8", 0.99)])
def test_full_checkpoint_768_row_decode_on_the_default_kernels(ckpt, kv, bound):
    """bf16 KV isolates the decode GEMMs (cosine >= 0.999); the default fp8
    KV cache adds e4m3 rounding of every cached key / value (>= 0.99)."""
    m = _load(ckpt, max_batch=512, max_rows=768, max_seq=512, kv_dtype=kv)
    assert m.use_tgemm and m.tg_head
    g = torch.Generator().manual_seed(2)
    base = _prompts(1, g)[0][:60]
    n_slots = 512
    # 8 distinct prompts over the slots, prefilled in batches
    prompts = [base[:30] + _prompts(1, g)[0][1:31] for _ in range(8)]
    for b in range(0, n_slots, 64):
        m.prefill_batch([(prompts[s % 8], s, 0) for s in range(b, b + 64)])
    rows = 768
    nxt = [int(t) for t in torch.randint(0, V - 256, (8,), generator=g)]
    # rows 0..511: every slot's next token; 512..767: jump rows of slots 0..255 one position further
    tk = torch.tensor([nxt[r % 8] if r < n_slots else nxt[(r - n_slots) % 8] for r in range(rows)],
                      dtype=torch.int32, device="cuda")
    sl = torch.tensor([r % n_slots for r in range(rows)], dtype=torch.int32, device="cuda")
    ps = torch.tensor([60 + (r // n_slots) for r in range(rows)], dtype=torch.int32, device="cuda")
    tk[n_slots:] = tk[:rows - n_slots]  # a jump row repeats its slot's token at the next position
    logits = m.decode(tk, sl, ps).float()
    coss = []
    for r in (0, 3, 7):
        ref = m.reference_logits(prompts[r % 8] + [nxt[r % 8]])[-1].float()
        coss.append(_cos(logits[r], ref))
    print(f"768-row decode ({kv} KV) logit cosine", [round(c, 5) for c in coss])
    assert min(coss) >= bound, coss
    # the fused head + masked argmax selects what the logits' argmax does
    masks = torch.full((1, (V + 31) // 32), -1, dtype=torch.int32, device="cuda")
    midx = torch.zeros(rows, dtype=torch.int32, device="cuda")
    last = torch.zeros(rows, dtype=torch.int32, device="cuda")
    src = torch.full((rows,), -1, dtype=torch.int32, device="cuda")
    lg, ids = m.decode_select_gather(tk, src, last, sl, ps, masks, midx)
    assert lg is None
    agree = (ids.cpu().long() == logits.argmax(-1).cpu()).float().mean().item()
    assert agree > 0.97, agree


def test_full_checkpoint_mxfp8_prefill_gate(ckpt):
    """MXFP8 prefill (e4m3 weights with per-row scales x MXFP8 activations) on
    trained-like weights vs fp32: the numbers that decide whether a loaded
    checkpoint may use it (LocalLM.load_safetensors, prefill_dtype auto)."""
    m = _load(ckpt, max_batch=16, max_rows=256, max_seq=1024, kv_dtype="bf16", prefill_dtype="fp8")
    assert m.prefill_fp8
    g = torch.Generator().manual_seed(3)
    prompts = _prompts(12, g)
    got = m.prefill_batch([(p, s, 0) for s, p in enumerate(prompts)]).float()
    coss, agree = [], 0
    for s, p in enumerate(prompts):
        ref = m.reference_logits(p)[-1].float()
        coss.append(_cos(got[s], ref))
        agree += int(got[s].argmax()) == int(ref.argmax())
    print("mxfp8 prefill logit cosine", [round(c, 5) for c in coss], "top-1", agree, "/", len(prompts))
    from dmcp.models.llm import MXFP8_CHECKPOINT_GATE
    passes = min(coss) >= MXFP8_CHECKPOINT_GATE["cosine"] and agree >= MXFP8_CHECKPOINT_GATE["top1"] * len(prompts)
    # a loaded checkpoint's prefill_dtype="auto" resolves to fp8 exactly when the gate passes
    # (measured round 6: cosine 0.89-0.93, top-1 3 / 12 -> bf16)
    m_auto = _load(ckpt, max_batch=4, max_rows=64, max_seq=256, kv_dtype="bf16")
    assert m_auto.prefill_fp8 == passes, (coss, agree)
