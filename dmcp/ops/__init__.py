"""Device ops for the local enrichment model.

GPU (HIP) tensors run the hand-written gfx950 kernels of ``dmcp/ops/csrc``
(:mod:`dmcp.ops.hip`, loaded from the in-tree ``_hipops.so``; a missing
library is an error, never a silent fallback).  CPU tensors run the fp32
PyTorch references of :mod:`dmcp.ops.reference` -- that path exists for
GPU-less unit tests, and only for the ops below that have one; the fused /
weight-streaming GEMMs are GPU-only and are re-exported from :mod:`.hip`.

Launch limits and plans (row limits, split counts, workspaces) are defined
once, in :mod:`.hip`, next to the kernels they describe.
"""
from __future__ import annotations

from . import hip, reference
from .hip import (FUSED_MAX_ROWS, PREFIX_MFMA_MAX_SPLITS, WGEMM_MAX_ROWS, decode_workspace,  # noqa: F401
                  fused_linear_norm, fused_rope_kv, fused_swiglu, lm_head_supported, lm_head_workspace,
                  prefill_supported, wgemm_resid_norm, wgemm_rope_kv, wgemm_swiglu, wgemm_workspace)
from .hip import (PGEMM_TILE_N, WMX_MAX_ROWS, pgemm_supported, wgemm_mx_resid_norm, wgemm_mx_rope_kv,  # noqa: F401
                  wgemm_mx_swiglu, wmx_plan)
from .hip import (TGEMM_MAX_ROWS, tgemm_lm_head_argmax, tgemm_resid_norm, tgemm_rope_kv, tgemm_swiglu,  # noqa: F401
                  wgemm)
from .reference import SharedPrefix, mx_dequant, quantize_weight, rope_tables, weight_dequant  # noqa: F401


def _on(t):
    """The implementation for tensor ``t``'s device."""
    return hip if t.is_cuda else reference


# ops with an fp32 CPU reference: the first tensor's device picks the kernel
def add_rmsnorm(x, weight, eps, residual=None, out=None):
    return _on(x).add_rmsnorm(x, weight, eps, residual, out)


def rope_kv(qkv, pos, slot, cos_sin, k_cache, v_cache, n_q_heads, q_out=None):
    return _on(qkv).rope_kv(qkv, pos, slot, cos_sin, k_cache, v_cache, n_q_heads, q_out)


def decode_attention(q, k_cache, v_cache, slot, seq_len, scale, workspace=None, chunk: int = 256, out=None,
                     prefix=None, splits=None, fork=None):
    if q.is_cuda:
        return hip.decode_attention(q, k_cache, v_cache, slot, seq_len, scale, workspace, chunk, out, prefix, splits,
                                    fork)
    return reference.decode_attention(q, k_cache, v_cache, slot, seq_len, scale, workspace, chunk, out, prefix, fork)


def prefill_attention(q, k_cache, v_cache, slot, start, prefix_slot=None, prefix_len=0, scale=1.0, out=None,
                      variant=0, nsplit=0):
    """Causal prefill/extend attention of one sequence, shared prefix read in place."""
    return _on(q).prefill_attention(q, k_cache, v_cache, slot, start, prefix_slot, prefix_len, scale, out, variant,
                                    nsplit)


def prefill_attention_varlen(q, k_cache, v_cache, offsets, slots, starts, prefix_slot=None, prefix_lens=None,
                             scale=1.0, out=None):
    return _on(q).prefill_attention_varlen(q, k_cache, v_cache, offsets, slots, starts, prefix_slot, prefix_lens,
                                           scale, out)


def silu_mul(gate_up, out=None):
    return _on(gate_up).silu_mul(gate_up, out)


def masked_argmax(logits, mask=None, vocab=None, out=None, mask_idx=None):
    return _on(logits).masked_argmax(logits, mask, vocab, out, mask_idx)


def lm_head_argmax(x, w, masks, mask_idx, out=None, workspace=None):
    """Grammar-masked greedy ids of the LM head (the logits never exist on the GPU path)."""
    return _on(x).lm_head_argmax(x, w, masks, mask_idx, out, workspace)


def embedding(table, ids, out=None):
    return _on(table).embedding(table, ids, out)


def decode_embed_norm(table, tokens, positions, weight, eps, src=None, last_ids=None, mask_idx=None, mask_alt=None,
                      alt_token: int = -1):
    """(resid, h, seq_len) of a decode step: each row's token (``last_ids[src]``
    where ``src >= 0``), its embedding, its first RMSNorm, its length; a
    gathered ``alt_token`` switches that row's grammar mask to ``mask_alt``."""
    return _on(table).decode_embed_norm(table, tokens, positions, weight, eps, src, last_ids, mask_idx, mask_alt,
                                        alt_token)


# GPU-only fused GEMM with a shape-dependent default
def fused_resid(x, w, residual, wk: int = 0):
    """residual += x . w^T in one gfx950 kernel; K-split waves by K."""
    return hip.fused_resid(x, w, residual, wk or (16 if x.shape[1] >= 4096 else 8))


def decode_plan(rows, n_kv_heads, max_seq, kv_dtype: str = "bf16"):
    """(chunk, splits) of the per-row decode attention (:func:`dmcp.ops.hip.decode_plan`).
    An fp8 cache halves the bytes per key, so fewer, longer splits keep the
    same bytes in flight: 2,048 target waves instead of 4,096 (fp8 step 2.35
    -> 2.30 ms at 78 rows, 5.54 -> 5.36 at 320; bf16 2.84 vs 2.94 the other
    way -- profiles/decode_target_waves_r2.txt)."""
    return hip.decode_plan(rows, n_kv_heads, max_seq, target_waves=2048 if kv_dtype == "fp8" else 4096)


# MXFP8 prefill path (csrc/pgemm.hip); CPU tensors run the fp32 references
def mx_quant(x, q=None, s=None):
    return _on(x).mx_quant(x, q, s)


def rmsnorm_mx(resid, weight, eps, add=None, q=None, s=None):
    return _on(resid).rmsnorm_mx(resid, weight, eps, add, q, s)


def pgemm(aq, as_, wq, ws, out=None):
    return _on(aq).pgemm(aq, as_, wq, ws, out)


def pgemm_resid(aq, as_, wq, ws, resid):
    return _on(aq).pgemm_resid(aq, as_, wq, ws, resid)


def pgemm_swiglu(aq, as_, wq, ws, q=None, s=None):
    return _on(aq).pgemm_swiglu(aq, as_, wq, ws, q, s)


def pgemm_qkv(aq, as_, wq, ws, pos, slot, cos_sin, k_cache, v_cache, n_q_heads, q_out=None):
    return _on(aq).pgemm_qkv(aq, as_, wq, ws, pos, slot, cos_sin, k_cache, v_cache, n_q_heads, q_out)
