"""Plain-PyTorch fp32 reference implementations of every HIP op.

Used (a) by the numerics tests, which compare each gfx950 kernel against
these, and (b) for CPU tensors (unit tests on the GPU-less build host).
Signatures mirror :mod:`dmcp.ops.hip`.
"""
from __future__ import annotations

from typing import NamedTuple, Optional

import torch


def add_rmsnorm(x: torch.Tensor, weight: torch.Tensor, eps: float, residual: Optional[torch.Tensor] = None,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
    h = x
    if residual is not None:
        h = (x.float() + residual.float()).to(x.dtype)
        residual.copy_(h)
    hf = h.float()
    y = hf * torch.rsqrt(hf.pow(2).mean(-1, keepdim=True) + eps) * weight.float()
    y = y.to(x.dtype)
    if out is not None:
        out.copy_(y)
        return out
    return y


# FP8 KV cache: uint8 tensors holding OCP e4m3fn bytes (unit scale, saturated)
FP8_MAX = 448.0


def kv_float(t: torch.Tensor) -> torch.Tensor:
    """Cache values as fp32 (bf16 caches, or fp8 e4m3 caches stored as uint8)."""
    if t.dtype == torch.uint8:
        return t.view(torch.float8_e4m3fn).float()
    return t.float()


def kv_encode(x: torch.Tensor, cache_dtype: torch.dtype) -> torch.Tensor:
    """Values in a cache's storage format (bf16, or saturated e4m3 bytes)."""
    if cache_dtype == torch.uint8:
        return x.float().clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn).view(torch.uint8)
    return x.to(cache_dtype)


def rope_tables(max_pos: int, head_dim: int, theta: float = 10000.0, device=None) -> torch.Tensor:
    """[max_pos, D/2, 2] float32 (cos, sin) -- viewed as float2 by the kernel."""
    half = head_dim // 2
    inv = 1.0 / (theta ** (torch.arange(0, half, dtype=torch.float64) / half))
    ang = torch.arange(max_pos, dtype=torch.float64)[:, None] * inv[None, :]
    return torch.stack([ang.cos(), ang.sin()], dim=-1).to(torch.float32).to(device)


def apply_rope(x: torch.Tensor, pos: torch.Tensor, cos_sin: torch.Tensor) -> torch.Tensor:
    """x [T, H, D] -> rotate-half RoPE at positions pos [T] (fp32 math)."""
    D = x.shape[-1]
    half = D // 2
    cs = cos_sin[pos.long().clamp(0, cos_sin.shape[0] - 1)].to(x.device)  # [T, half, 2]
    c = cs[..., 0][:, None, :]
    s = cs[..., 1][:, None, :]
    xf = x.float()
    x1, x2 = xf[..., :half], xf[..., half:]
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1)


def rope_kv(qkv: torch.Tensor, pos: torch.Tensor, slot: torch.Tensor, cos_sin: torch.Tensor,
            k_cache: torch.Tensor, v_cache: torch.Tensor, n_q_heads: int, q_out: Optional[torch.Tensor] = None
            ) -> torch.Tensor:
    S, Hkv, MAXS, D = k_cache.shape
    T = qkv.shape[0]
    x = qkv.view(T, n_q_heads + 2 * Hkv, D)
    q = apply_rope(x[:, :n_q_heads], pos, cos_sin).to(qkv.dtype)
    k = apply_rope(x[:, n_q_heads:n_q_heads + Hkv], pos, cos_sin).to(qkv.dtype)
    v = x[:, n_q_heads + Hkv:]
    for t in range(T):
        p, s = int(pos[t]), int(slot[t])
        if 0 <= p < MAXS and 0 <= s < S:
            k_cache[s, :, p] = kv_encode(k[t], k_cache.dtype)
            v_cache[s, :, p] = kv_encode(v[t], v_cache.dtype)
    if q_out is not None:
        q_out.copy_(q)
        return q_out
    return q


class SharedPrefix(NamedTuple):
    """Keys/values shared by the rows of a decode step (cascade decoding):
    ``k`` / ``v`` [Hkv, MAXS, D] (the prefix slot of the caches),
    ``length`` int32 [1] on the device (0 = no prefix) and ``rows`` (int32
    [B], optional: 0 = this row does not use the prefix)."""
    k: torch.Tensor
    v: torch.Tensor
    length: torch.Tensor
    rows: Optional[torch.Tensor] = None


def decode_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, slot: torch.Tensor,
                     seq_len: torch.Tensor, scale: float, workspace=None, chunk: int = 256,
                     out: Optional[torch.Tensor] = None, prefix: Optional[SharedPrefix] = None,
                     fork: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``fork`` [S, 2] (parent slot, end): keys below ``end`` of a row whose
    slot has a parent come from the parent's slot (a method branch reading
    its class head's KV in place)."""
    B, Hq, D = q.shape
    S, Hkv, MAXS, _ = k_cache.shape
    G = Hq // Hkv
    P = int(prefix.length.reshape(-1)[0]) if prefix is not None else 0
    res = torch.zeros((B, Hq, D), dtype=torch.float32, device=q.device)
    for b in range(B):
        s, L = int(slot[b]), min(int(seq_len[b]), MAXS)
        if not (0 <= s < S) or L <= 0:
            continue
        k = kv_float(k_cache[s, :, :L])  # [Hkv, L, D]
        v = kv_float(v_cache[s, :, :L])
        if fork is not None:
            ps, fe = int(fork[s, 0]), min(int(fork[s, 1]), L)
            if fe > 0 and 0 <= ps < S and ps != s:
                k = torch.cat([kv_float(k_cache[ps, :, :fe]), k[:, fe:]], dim=1)
                v = torch.cat([kv_float(v_cache[ps, :, :fe]), v[:, fe:]], dim=1)
        if P > 0 and (prefix.rows is None or int(prefix.rows[b]) != 0):  # the first P keys: the shared prefix
            k = torch.cat([kv_float(prefix.k[:, :P]), k[:, P:]], dim=1)
            v = torch.cat([kv_float(prefix.v[:, :P]), v[:, P:]], dim=1)
        qb = q[b].float().view(Hkv, G, D)
        att = torch.einsum("hgd,hld->hgl", qb, k) * scale
        p = torch.softmax(att, dim=-1)
        res[b] = torch.einsum("hgl,hld->hgd", p, v).reshape(Hq, D)
    y = res.to(q.dtype)
    if out is not None:
        out.copy_(y)
        return out
    return y


def prefill_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, slot: int, start: int,
                      prefix_slot: Optional[int] = None, prefix_len: int = 0, scale: float = 1.0,
                      out: Optional[torch.Tensor] = None, variant: int = 0, nsplit: int = 0) -> torch.Tensor:
    """q [T, Hq, D] at positions [start, start+T) of ``slot``; every query
    sees the keys at or before its position.  Keys [0, prefix_len) come from
    ``prefix_slot``, the rest from ``slot``.  fp32 math, returns [T, Hq, D]."""
    T, Hq, D = q.shape
    Hkv = k_cache.shape[1]
    G = Hq // Hkv
    L = start + T
    k = kv_float(k_cache[slot, :, :L])
    v = kv_float(v_cache[slot, :, :L])
    if prefix_len > 0:
        k = torch.cat([kv_float(k_cache[prefix_slot, :, :prefix_len]), k[:, prefix_len:]], dim=1)
        v = torch.cat([kv_float(v_cache[prefix_slot, :, :prefix_len]), v[:, prefix_len:]], dim=1)
    qf = q.float().view(T, Hkv, G, D)
    att = torch.einsum("thgd,hld->hgtl", qf, k) * scale  # [Hkv, G, T, L]
    pos = torch.arange(start, L, device=q.device)[:, None]
    att = att.masked_fill(torch.arange(L, device=q.device)[None, :] > pos, float("-inf"))
    y = torch.einsum("hgtl,hld->thgd", torch.softmax(att, dim=-1), v).reshape(T, Hq, D).to(q.dtype)
    if out is not None:
        out.copy_(y)
        return out
    return y


def prefill_attention_varlen(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, offsets, slots, starts,
                             prefix_slot: Optional[int] = None, prefix_lens=None, scale: float = 1.0,
                             out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Several sequences' prefill in one packed q [Ttot, Hq, D]: sequence i
    is rows [offsets[i], offsets[i+1]) at positions [starts[i], ...) of
    ``slots[i]``, keys [0, prefix_lens[i]) read from ``prefix_slot``.
    fp32 math per sequence (:func:`prefill_attention`)."""
    out = torch.empty_like(q) if out is None else out
    for i in range(len(slots)):
        a, b = int(offsets[i]), int(offsets[i + 1])
        P = int(prefix_lens[i]) if prefix_lens is not None else 0
        out[a:b] = prefill_attention(q[a:b], k_cache, v_cache, int(slots[i]), int(starts[i]),
                                     prefix_slot if P else None, P, scale)
    return out


def silu_mul(gate_up: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    I = gate_up.shape[-1] // 2
    g, u = gate_up[..., :I].float(), gate_up[..., I:].float()
    y = (torch.nn.functional.silu(g) * u).to(gate_up.dtype)
    if out is not None:
        out.copy_(y)
        return out
    return y


def masked_argmax(logits: torch.Tensor, mask: Optional[torch.Tensor] = None, vocab: Optional[int] = None,
                  out: Optional[torch.Tensor] = None, mask_idx: Optional[torch.Tensor] = None) -> torch.Tensor:
    B, ld = logits.shape
    V = vocab or ld
    x = logits[:, :V].float().clone()
    if mask is not None and mask_idx is not None:
        mask = mask[mask_idx.long().clamp(0, mask.shape[0] - 1)]
    if mask is not None:
        idx = torch.arange(V, device=logits.device)
        words = mask.to(torch.int64)[:, idx // 32]
        bits = (words >> (idx % 32)) & 1
        x[bits == 0] = float("-inf")
    ids = torch.argmax(x, dim=-1).to(torch.int32)  # first index among ties
    if out is not None:
        out.copy_(ids)
        return out
    return ids


def lm_head_argmax(x: torch.Tensor, w: torch.Tensor, masks: torch.Tensor, mask_idx: torch.Tensor,
                   out: Optional[torch.Tensor] = None, workspace=None) -> torch.Tensor:
    """The fused LM head + masked argmax's definition: F.linear then masked_argmax."""
    logits = (x.float() @ w.float().t()).to(torch.bfloat16)
    return masked_argmax(logits, masks, w.shape[0], out, mask_idx)


def embedding(table: torch.Tensor, ids: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    y = table[ids.long().clamp(0, table.shape[0] - 1)]
    if out is not None:
        out.copy_(y)
        return out
    return y


def decode_embed_norm(table: torch.Tensor, tokens: torch.Tensor, positions: torch.Tensor,
                      weight: Optional[torch.Tensor], eps: float, src: Optional[torch.Tensor] = None,
                      last_ids: Optional[torch.Tensor] = None, mask_idx: Optional[torch.Tensor] = None,
                      mask_alt: Optional[torch.Tensor] = None, alt_token: int = -1) -> tuple:
    """(resid, h, seq_len) of the decode step's first op (see the HIP kernel);
    ``mask_alt``: gathered rows whose token is ``alt_token`` switch
    ``mask_idx`` (in place) to ``mask_alt`` where that is >= 0."""
    toks = tokens
    if src is not None:
        s = src.long()
        gathered = last_ids.long()[s.clamp(0, last_ids.numel() - 1)].to(tokens.dtype)
        toks = torch.where(s >= 0, gathered, tokens)
        if mask_alt is not None:
            sw = (s >= 0) & (gathered == alt_token) & (mask_alt >= 0)
            mask_idx.copy_(torch.where(sw, mask_alt, mask_idx))
    resid = embedding(table, toks)
    h = add_rmsnorm(resid, weight, eps) if weight is not None else None
    return resid, h, positions + 1


# ---- MXFP8 prefill GEMMs (csrc/pgemm.hip): activations as e4m3 bytes with one
# power-of-two (E8M0) scale per 32 consecutive elements of a row, weights as
# e4m3 bytes with one fp32 scale per output row.
_INV_FP8_MAX = torch.tensor(1.0 / FP8_MAX, dtype=torch.float32)


def mx_quant(x: torch.Tensor, q: Optional[torch.Tensor] = None, s: Optional[torch.Tensor] = None) -> tuple:
    """[M, K] (K % 32 == 0) -> (q uint8 [M, K] e4m3, s uint8 [M, K / 32] E8M0):
    block exponent e = the smallest with max|x| / 2^e <= 448, q = x / 2^e."""
    M, K = x.shape
    xf = x.float().reshape(M, K // 32, 32)
    amax = xf.abs().amax(-1)
    _, e = torch.frexp(amax * _INV_FP8_MAX.to(x.device))
    e = torch.where(amax > 0, e, torch.zeros_like(e)).clamp(-127, 127)
    qv = torch.ldexp(xf, (-e)[..., None].to(torch.float32))
    qb = qv.clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn).view(torch.uint8).reshape(M, K)
    sb = (e + 127).to(torch.uint8)
    if q is not None:
        q.copy_(qb)
        s.copy_(sb)
        return q, s
    return qb, sb


def mx_dequant(q: torch.Tensor, s: torch.Tensor) -> torch.Tensor:
    """fp32 values of an MXFP8 tensor."""
    M, K = q.shape
    v = q.view(torch.float8_e4m3fn).float().reshape(M, K // 32, 32)
    return torch.ldexp(v, (s.to(torch.int32) - 127)[..., None].to(torch.float32)).reshape(M, K)


def quantize_weight(w: torch.Tensor) -> tuple:
    """[N, K] -> (e4m3 bytes [N, K], fp32 scale [N]): per-output-row scale max|w| / 448."""
    wf = w.float()
    sc = wf.abs().amax(-1) / FP8_MAX
    sc = torch.where(sc > 0, sc, torch.ones_like(sc))
    wq = (wf / sc[:, None]).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn).view(torch.uint8)
    return wq.contiguous(), sc.to(torch.float32).contiguous()


def weight_dequant(wq: torch.Tensor, ws: torch.Tensor) -> torch.Tensor:
    return wq.view(torch.float8_e4m3fn).float() * ws[:, None].float()


def _pgemm_f32(aq, as_, wq, ws) -> torch.Tensor:
    return mx_dequant(aq, as_) @ weight_dequant(wq, ws).t()


def rmsnorm_mx(resid: torch.Tensor, weight: torch.Tensor, eps: float, add: Optional[torch.Tensor] = None,
               q: Optional[torch.Tensor] = None, s: Optional[torch.Tensor] = None) -> tuple:
    """resid += add (bf16, in place); RMSNorm(resid) * weight as MXFP8."""
    if add is not None:
        resid.copy_((resid.float() + add.float()).to(resid.dtype))
    hf = resid.float()
    y = hf * torch.rsqrt(hf.pow(2).mean(-1, keepdim=True) + eps) * weight.float()
    return mx_quant(y, q, s)


def pgemm(aq, as_, wq, ws, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    y = _pgemm_f32(aq, as_, wq, ws).to(torch.bfloat16)
    if out is not None:
        out.copy_(y)
        return out
    return y


def pgemm_resid(aq, as_, wq, ws, resid: torch.Tensor) -> torch.Tensor:
    y = _pgemm_f32(aq, as_, wq, ws).to(torch.bfloat16)
    resid.copy_((resid.float() + y.float()).to(resid.dtype))
    return resid


def pgemm_swiglu(aq, as_, wq, ws, q: Optional[torch.Tensor] = None, s: Optional[torch.Tensor] = None) -> tuple:
    """silu(gate) * up of the stacked [gate; up] weight, as MXFP8 [M, I]."""
    gu = _pgemm_f32(aq, as_, wq, ws).to(torch.bfloat16).float()
    inter = gu.shape[1] // 2
    g, u = gu[:, :inter], gu[:, inter:]
    return mx_quant(g / (1.0 + torch.exp(-g)) * u, q, s)


def pgemm_qkv(aq, as_, wq, ws, pos, slot, cos_sin, k_cache, v_cache, n_q_heads: int,
              q_out: Optional[torch.Tensor] = None) -> torch.Tensor:
    qkv = _pgemm_f32(aq, as_, wq, ws).to(torch.bfloat16)
    return rope_kv(qkv, pos, slot, cos_sin, k_cache, v_cache, n_q_heads, q_out)
