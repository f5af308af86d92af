"""Device ops for the local enrichment model.

GPU (HIP) tensors run the hand-written gfx950 kernels of
``dmcp/ops/csrc/dmcp_kernels.hip`` (loaded from the in-tree ``_hipops.so``;
a missing library is an error, never a silent fallback).  CPU tensors run
the fp32 PyTorch references in :mod:`dmcp.ops.reference` -- that path only
exists for GPU-less unit tests.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import reference


def _hip():
    from . import hip
    return hip


def add_rmsnorm(x, weight, eps, residual=None, out=None):
    return (_hip() if x.is_cuda else reference).add_rmsnorm(x, weight, eps, residual, out)


def decode_chunk(rows, n_kv_heads, max_seq):
    """Keys per split-K work item for a decode step (see :func:`dmcp.ops.hip.decode_chunk`)."""
    from .hip import decode_chunk as _dc
    return _dc(rows, n_kv_heads, max_seq)


def decode_plan(rows, n_kv_heads, max_seq, kv_dtype: str = "bf16"):
    """(chunk, splits) of the per-row decode attention (see :func:`dmcp.ops.hip.decode_plan`).
    An fp8 cache halves the bytes per key, so fewer, longer splits keep the
    same bytes in flight: 2,048 target waves instead of 4,096 (fp8 step 2.35
    -> 2.30 ms at 78 rows, 5.54 -> 5.36 at 320; bf16 2.84 vs 2.94 the other
    way -- profiles/decode_target_waves_r2.txt)."""
    from .hip import decode_plan as _dp
    return _dp(rows, n_kv_heads, max_seq, target_waves=2048 if kv_dtype == "fp8" else 4096)


PREFIX_MFMA_MAX_SPLITS = 16  # shared-prefix key splits on the prefill kernel (dmcp.ops.hip)
FUSED_MAX_ROWS = 128  # row limit of the fused decode GEMMs (dmcp.ops.hip.FUSED_MAX_ROWS)


def fused_rope_kv(x, w, eps, pos, slot, cos_sin, k_cache, v_cache, n_q_heads, q_out=None):
    """RMSNorm -> QKV GEMM -> RoPE -> KV append in one gfx950 kernel (GPU only)."""
    return _hip().fused_rope_kv(x, w, eps, pos, slot, cos_sin, k_cache, v_cache, n_q_heads, q_out)


def fused_swiglu(x, w, eps, out=None):
    """RMSNorm -> gate/up GEMM -> SwiGLU in one gfx950 kernel (GPU only)."""
    return _hip().fused_swiglu(x, w, eps, out)


def fused_resid(x, w, residual, wk: int = 0):
    """residual += x . w^T in one gfx950 kernel (GPU only); K-split waves by K."""
    return _hip().fused_resid(x, w, residual, wk or (16 if x.shape[1] >= 4096 else 8))


WGEMM_MAX_ROWS = 512  # row limit of the weight-streaming GEMMs (dmcp.ops.hip.WGEMM_MAX_ROWS)


def wgemm_swiglu(x, w, out=None):
    """silu(x . w[:I]^T) * (x . w[I:]^T) on the weight-streaming gfx950 GEMM (GPU only, M <= 512)."""
    return _hip().wgemm_swiglu(x, w, out)


def wgemm_resid_norm(x, w, residual, norm_w, eps, workspace, out=None):
    """residual += bf16(x . w^T); returns RMSNorm(residual) * norm_w -- split-K
    weight-streaming GEMM + one fused reduce/residual/norm pass (GPU only)."""
    return _hip().wgemm_resid_norm(x, w, residual, norm_w, eps, workspace, out)


def wgemm_rope_kv(x, w, pos, slot, cos_sin, k_cache, v_cache, n_q_heads, workspace, q_out=None):
    """rope_kv(F.linear(x, w)) -- split-K weight-streaming GEMM + one reduction
    that applies RoPE and appends K/V to the cache (GPU only)."""
    return _hip().wgemm_rope_kv(x, w, pos, slot, cos_sin, k_cache, v_cache, n_q_heads, workspace, q_out)


def wgemm_workspace(rows, n_max, device):
    return _hip().wgemm_workspace(rows, n_max, device)


def fused_linear_norm(x, w, eps, out=None):
    """RMSNorm -> GEMM (bf16 out; the LM head) in one gfx950 kernel (GPU only)."""
    return _hip().fused_linear_norm(x, w, eps, out)


def decode_workspace(rows, n_heads, n_kv_heads, head_dim, max_seq, device, chunk: int = 256, prefix_slots: int = 0):
    """Split-K scratch of the decode-attention kernel (fp32 partials + max/sum)."""
    return _hip().decode_workspace(rows, n_heads, n_kv_heads, head_dim, max_seq, device, chunk, prefix_slots)


def rope_kv(qkv, pos, slot, cos_sin, k_cache, v_cache, n_q_heads, q_out=None):
    return (_hip() if qkv.is_cuda else reference).rope_kv(qkv, pos, slot, cos_sin, k_cache, v_cache, n_q_heads, q_out)


def decode_attention(q, k_cache, v_cache, slot, seq_len, scale, workspace=None, chunk: int = 256, out=None,
                     prefix=None, splits=None):
    if q.is_cuda:
        return _hip().decode_attention(q, k_cache, v_cache, slot, seq_len, scale, workspace, chunk, out, prefix,
                                       splits)
    return reference.decode_attention(q, k_cache, v_cache, slot, seq_len, scale, workspace, chunk, out, prefix)


def prefill_attention(q, k_cache, v_cache, slot, start, prefix_slot=None, prefix_len=0, scale=1.0, out=None,
                      variant=0, nsplit=0):
    """Causal prefill/extend attention of one sequence, shared prefix read in place."""
    return (_hip() if q.is_cuda else reference).prefill_attention(q, k_cache, v_cache, slot, start, prefix_slot,
                                                                  prefix_len, scale, out, variant, nsplit)


def prefill_attention_varlen(q, k_cache, v_cache, offsets, slots, starts, prefix_slot=None, prefix_lens=None,
                             scale=1.0, out=None):
    return (_hip() if q.is_cuda else reference).prefill_attention_varlen(
        q, k_cache, v_cache, offsets, slots, starts, prefix_slot, prefix_lens, scale, out)


def prefill_supported(n_heads, n_kv_heads, head_dim):
    from .hip import prefill_supported as _ps
    return _ps(n_heads, n_kv_heads, head_dim)


def silu_mul(gate_up, out=None):
    return (_hip() if gate_up.is_cuda else reference).silu_mul(gate_up, out)


def masked_argmax(logits, mask=None, vocab: Optional[int] = None, out=None, mask_idx=None):
    return (_hip() if logits.is_cuda else reference).masked_argmax(logits, mask, vocab, out, mask_idx)


def embedding(table, ids, out=None):
    return (_hip() if table.is_cuda else reference).embedding(table, ids, out)


rope_tables = reference.rope_tables
SharedPrefix = reference.SharedPrefix
