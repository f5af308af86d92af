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


def _by_device(name: str):
    """``name`` dispatched on its first tensor argument's device: the gfx950
    kernel (:mod:`.hip`) for GPU tensors, the fp32 reference for CPU ones.
    Both modules implement these ops with the same signature
    (tests/test_launch_plans.py::test_device_ops_share_one_signature); the
    GPU kernel's docstring is the op's."""
    k, r = getattr(hip, name), getattr(reference, name)

    def op(first, *args, **kw):
        return (k if first.is_cuda else r)(first, *args, **kw)
    op.__name__ = op.__qualname__ = name
    op.__doc__ = k.__doc__ or r.__doc__
    op.__wrapped__ = k  # inspect.signature reports the kernel's parameters
    return op


# ops with an fp32 CPU reference: norms, RoPE + KV append, prefill attention,
# SwiGLU, selection, embedding, the decode step's input gather + first norm,
# and the MXFP8 prefill path (csrc/pgemm.hip)
DEVICE_OPS = ("add_rmsnorm", "rope_kv", "prefill_attention", "prefill_attention_varlen", "silu_mul",
              "masked_argmax", "lm_head_argmax", "embedding", "decode_embed_norm", "mx_quant", "rmsnorm_mx",
              "pgemm", "pgemm_resid", "pgemm_swiglu", "pgemm_qkv")
for _name in DEVICE_OPS:
    globals()[_name] = _by_device(_name)
del _name


def decode_attention(q, k_cache, v_cache, slot, seq_len, scale, workspace=None, chunk: int = 256, out=None,
                     prefix=None, splits=None, fork=None):
    """Per-row decode attention; the CPU reference takes no split count."""
    if q.is_cuda:
        return hip.decode_attention(q, k_cache, v_cache, slot, seq_len, scale, workspace, chunk, out, prefix, splits,
                                    fork)
    return reference.decode_attention(q, k_cache, v_cache, slot, seq_len, scale, workspace, chunk, out, prefix, fork)


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
