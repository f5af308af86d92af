"""ctypes binding of the gfx950 kernel library + tensor-level wrappers.

Every wrapper validates dtype / device / contiguity / shapes on the host
*before* launching (a mis-shaped launch can fault the GPU), launches on
torch's current HIP stream (so calls compose with hipBLASLt GEMMs and can be
captured into hipGraphs) and raises on any non-zero hipError.

On a GPU box the library MUST load: :func:`lib` raises instead of silently
falling back to PyTorch.  CPU tensors are routed to :mod:`dmcp.ops.reference`
by :mod:`dmcp.ops` (CPU unit tests only).
"""
from __future__ import annotations

import ctypes
import math
import os
import threading
from typing import Optional

import numpy as np
import torch

from .build import TARGET, build

_lib = None
_lock = threading.Lock()
_vp = ctypes.c_void_p
_i = ctypes.c_int
_f = ctypes.c_float
ABI_VERSION = 17  # must match dmcp_abi_version() in csrc/dmcp_kernels.hip


class HipOpsError(RuntimeError):
    pass


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        # DMCP_HIPOPS_SO: another build of the same ABI (bench A/B of a kernel
        # change, scripts/hipops_ab.sh); the in-tree library otherwise
        path = os.environ.get("DMCP_HIPOPS_SO") or TARGET
        if not os.path.exists(path):
            if os.environ.get("DMCP_NO_AUTOBUILD") or path != TARGET:
                raise HipOpsError(f"HIP kernel library missing: {path}")
            path = build()
        L = ctypes.CDLL(path)
        sigs = {
            "dmcp_abi_version": ([], _i),
            "dmcp_lm_head_argmax": ([_vp, _vp, _vp, _vp, _i, _i, _vp, _vp, _i, _i, _i, _i, _vp], _i),
            "dmcp_add_rmsnorm": ([_vp, _vp, _vp, _vp, _i, _i, _f, _vp], _i),
            "dmcp_rope_kv": ([_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _vp], _i),
            "dmcp_decode_attention": ([_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _f,
                                       _vp, _vp, _vp, _i, _i, _vp, _vp, _vp], _i),
            "dmcp_kv_fork": ([_vp, _vp, _i, _i, _i, _i, _i, _i, _vp, _i, _i, _i, _vp], _i),
            "dmcp_pgemm_set_waves": ([_i], _i),
            "dmcp_pgemm_set_bk": ([_i], _i),
            "dmcp_wgemm_set_aux": ([_i], _i),
            "dmcp_pgemm_set_group": ([_i], _i),
            "dmcp_pgemm_set_areg": ([_i], _i),
            "dmcp_prefill_attention": ([_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _f, _i, _i,
                                        _i, _vp], _i),
            "dmcp_prefill_varlen": ([_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, ctypes.c_long, _f,
                                     _i, _vp], _i),
            "dmcp_silu_mul": ([_vp, _vp, _i, _i, _vp], _i),
            "dmcp_masked_argmax": ([_vp, _vp, _vp, _i, _vp, _i, _i, _i, _vp], _i),
            "dmcp_embedding": ([_vp, _vp, _vp, _i, _i, _i, _vp], _i),
            "dmcp_decode_embed_norm": ([_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _f, _vp, _vp,
                                        _i, _vp], _i),
            "dmcp_fused_gemm_max_rows": ([], _i),
            "dmcp_pgemm": ([_vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _vp], _i),
            "dmcp_pgemm_swiglu": ([_vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _vp], _i),
            "dmcp_pgemm_qkv": ([_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i,
                                _vp], _i),
            "dmcp_mx_quant": ([_vp, _vp, _vp, _i, _i, _vp], _i),
            "dmcp_rmsnorm_mx": ([_vp, _vp, _vp, _vp, _vp, _i, _i, _f, _vp], _i),
            "dmcp_mx_probe": ([_vp, _vp, _vp, _vp, _vp, _vp], _i),
            "dmcp_wgemm_mx": ([_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _vp], _i),
            "dmcp_reduce_resid_norm_mx": ([_vp, _i, _vp, _vp, _vp, _vp, _i, _i, _f, _vp], _i),
            "dmcp_reduce_resid_norm": ([_vp, _i, _vp, _vp, _vp, _i, _i, _f, _vp], _i),
            "dmcp_reduce_rope_kv": ([_vp, _i, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _vp], _i),
            "dmcp_wgemm": ([_vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _vp], _i),
            "dmcp_tgemm": ([_vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _vp, _vp, _i, _i, _vp, _vp], _i),
            "dmcp_tgemm_probe": ([_i, _vp, _vp, _vp, _i, _i, _i, _i, _i, _vp], _i),
            "dmcp_wgemm_resid_norm": ([_vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _f, _vp], _i),
            "dmcp_wgemm_rope_kv": ([_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _i,
                                    _i, _i, _vp], _i),
            "dmcp_fused_gemm": ([_i, _i, _vp, _vp, _vp, _i, _i, _i, _f, _i, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i,
                                 _i, _i, _i, _i, _vp], _i),
        }
        for name, (args, res) in sigs.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        if L.dmcp_abi_version() != ABI_VERSION:
            raise HipOpsError("HIP kernel library ABI mismatch; rebuild with python -m dmcp.ops.build")
        _lib = L
        return _lib


def loaded_path() -> Optional[str]:
    return (os.environ.get("DMCP_HIPOPS_SO") or TARGET) if _lib is not None else None


def _stream() -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ptr(t: Optional[torch.Tensor]) -> ctypes.c_void_p:
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def _check(rc: int, name: str) -> None:
    if rc != 0:
        raise HipOpsError(f"{name} failed with hipError {rc}")


def _req(t: torch.Tensor, dtype: torch.dtype, name: str) -> None:
    if not t.is_cuda:
        raise HipOpsError(f"{name}: tensor must be on the GPU")
    if t.dtype != dtype:
        raise HipOpsError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise HipOpsError(f"{name}: tensor must be contiguous")


KV_DTYPES = (torch.bfloat16, torch.uint8)  # bf16 or fp8 e4m3 bytes (dmcp.ops.reference.kv_encode)


def _req_kv(k_cache: torch.Tensor, v_cache: torch.Tensor, name: str) -> int:
    """KV caches: same shape, both bf16 or both fp8 (uint8 storage); returns the kv8 flag."""
    if k_cache.dtype not in KV_DTYPES or v_cache.dtype != k_cache.dtype:
        raise HipOpsError(f"{name}: KV caches must both be bf16 or both fp8 (uint8), got {k_cache.dtype} / "
                          f"{v_cache.dtype}")
    _req(k_cache, k_cache.dtype, f"{name}.k_cache")
    _req(v_cache, v_cache.dtype, f"{name}.v_cache")
    if v_cache.shape != k_cache.shape:
        raise HipOpsError(f"{name}: k/v cache shapes differ")
    return int(k_cache.dtype == torch.uint8)


def _req_out(t: torch.Tensor, dtype: torch.dtype, numel: int, name: str) -> None:
    """A caller-supplied output buffer: same checks as :func:`_req` plus room
    for the ``numel`` elements the kernel writes (an undersized buffer would be
    an out-of-bounds device write)."""
    _req(t, dtype, name)
    if t.numel() < numel:
        raise HipOpsError(f"{name}: buffer holds {t.numel()} elements, the kernel writes {numel}")


# ---------------------------------------------------------------- wrappers
def add_rmsnorm(x: torch.Tensor, weight: torch.Tensor, eps: float, residual: Optional[torch.Tensor] = None,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
    H = x.shape[-1]
    rows = x.numel() // H
    _req(x, torch.bfloat16, "add_rmsnorm.x")
    _req(weight, torch.bfloat16, "add_rmsnorm.weight")
    if weight.numel() != H or H % 8 or H > 8192:
        raise HipOpsError(f"add_rmsnorm: unsupported hidden size {H}")
    if residual is not None:
        _req(residual, torch.bfloat16, "add_rmsnorm.residual")
        if residual.shape != x.shape:
            raise HipOpsError("add_rmsnorm: residual shape mismatch")
    out = torch.empty_like(x) if out is None else out
    _req_out(out, torch.bfloat16, rows * H, "add_rmsnorm.out")
    if rows == 0:
        return out
    _check(lib().dmcp_add_rmsnorm(_ptr(x), _ptr(residual), _ptr(weight), _ptr(out), rows, H, float(eps), _stream()),
           "dmcp_add_rmsnorm")
    return out


def rope_kv(qkv: torch.Tensor, pos: torch.Tensor, slot: torch.Tensor, cos_sin: torch.Tensor,
            k_cache: torch.Tensor, v_cache: torch.Tensor, n_q_heads: int, q_out: Optional[torch.Tensor] = None
            ) -> torch.Tensor:
    """k_cache/v_cache: [S, Hkv, MAXS, D]; returns q [T, Hq, D]."""
    S, Hkv, MAXS, D = k_cache.shape
    T = qkv.shape[0]
    _req(qkv, torch.bfloat16, "rope_kv.qkv")
    kv8 = _req_kv(k_cache, v_cache, "rope_kv")
    _req(pos, torch.int32, "rope_kv.pos")
    _req(slot, torch.int32, "rope_kv.slot")
    _req(cos_sin, torch.float32, "rope_kv.cos_sin")
    if v_cache.shape != k_cache.shape or qkv.shape[1] != (n_q_heads + 2 * Hkv) * D or D % 16:
        raise HipOpsError("rope_kv: shape mismatch")
    # cos_sin is [max_pos, D/2, 2] (cos, sin) -- read as float2 by the kernel
    if pos.numel() != T or slot.numel() != T or cos_sin.dim() != 3 or tuple(cos_sin.shape[1:]) != (D // 2, 2) \
            or cos_sin.shape[0] < 1:
        raise HipOpsError(f"rope_kv: pos/slot/cos_sin shape mismatch (cos_sin {tuple(cos_sin.shape)}, D={D})")
    max_pos = cos_sin.shape[0]
    if q_out is None:
        q_out = torch.empty((T, n_q_heads, D), dtype=torch.bfloat16, device=qkv.device)
    _req_out(q_out, torch.bfloat16, T * n_q_heads * D, "rope_kv.q_out")
    _check(lib().dmcp_rope_kv(_ptr(qkv), _ptr(pos), _ptr(slot), _ptr(cos_sin), _ptr(q_out), _ptr(k_cache),
                              _ptr(v_cache), T, n_q_heads, Hkv, D, MAXS, max_pos, S, kv8, _stream()), "dmcp_rope_kv")
    return q_out


def decode_splits(max_seq: int, chunk: int = 256) -> int:
    return max(1, math.ceil(max_seq / chunk))


def decode_chunk(rows: int, n_kv_heads: int, max_seq: int, target_items: int = 2048) -> int:
    """Keys per split-K work item for a decode step of ``rows`` query rows
    (the round-1 heuristic, kept for callers that pass only ``chunk``;
    :func:`decode_plan` is what the model uses)."""
    for chunk in (1024, 512):
        if rows * n_kv_heads * decode_splits(max_seq, chunk) >= target_items:
            return chunk
    return 256


def decode_plan(rows: int, n_kv_heads: int, max_seq: int, target_waves: int = 4096,
                min_chunk: int = 256) -> tuple:
    """(chunk, splits) for a decode step of ``rows`` query rows.

    The per-row kernel is bound by HBM latency x bytes in flight: one wave
    per (row, kv head, split) keeps one 32-key tile of K/V loads in flight,
    so the step needs ~16 busy waves per CU (4 per SIMD at the kernel's 128
    VGPRs; 4096 on 256 CUs).  Each row's keys are cut into at most
    ``splits`` EQUAL parts of >= ``min_chunk`` keys (rounded to 32-key
    tiles, in-kernel from the live length), instead of full fixed-size
    chunks plus a short remainder that left most waves idle at the end
    (measured: 1024-key chunks reached 42 % of the copy rate at B = 78,
    L = 2,500 -- profiles/decode_step_r2*).  More parts for the engine's long
    rows (up to 8 of >= 256 / 512 keys) measured slower on both presets
    (profiles/decode_split_engine_ab_r6.txt).  ``DMCP_DECODE_MIN_CHUNK`` /
    ``DMCP_DECODE_MIN_SPLITS`` override (A/B)."""
    min_chunk = int(os.environ.get("DMCP_DECODE_MIN_CHUNK", min_chunk))  # A/B overrides
    splits = max(1, -(-target_waves // max(1, rows * n_kv_heads)), int(os.environ.get("DMCP_DECODE_MIN_SPLITS", 1)))
    return min_chunk, min(splits, decode_splits(max_seq, min_chunk))


def decode_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, slot: torch.Tensor,
                     seq_len: torch.Tensor, scale: float, workspace: Optional[tuple] = None,
                     chunk: int = 256, out: Optional[torch.Tensor] = None,
                     prefix: Optional["SharedPrefix"] = None, splits: Optional[int] = None,
                     fork: Optional[torch.Tensor] = None) -> torch.Tensor:
    """q [B, Hq, D]; caches [S, Hkv, MAXS, D]; slot/seq_len int32 [B].

    ``fork`` (int32 [S, 2], optional): per slot (parent slot, end) -- a
    method branch reads its keys below ``end`` from its class head's slot in
    place (no copy); end 0 = no parent.

    Each row's keys (after the shared prefix) are split into at most
    ``splits`` equal parts of >= ``chunk`` keys (default: as many as
    ``MAXS / chunk``, i.e. parts of <= ``chunk`` keys); see :func:`decode_plan`.

    ``prefix``: the first ``*prefix.length`` keys of every row are the shared
    prefix (``prefix.k`` / ``prefix.v`` [Hkv, MAXS, D], the prefix slot),
    attended by the MFMA prefill kernel in prefix mode (every prefix key read
    once per 32 queries, :func:`prefix_mfma_splits` key splits); the per-row
    kernel covers the keys after it.  The length lives in device memory, so
    a captured graph follows prefix changes (0 = no prefix).  ``prefix.rows``
    (int32 [B], optional): rows marked 0 do not use the prefix -- all their
    keys are in their own slot (a sequence of another project, admitted while
    this prefix is resident)."""
    B, Hq, D = q.shape
    S, Hkv, MAXS, Dk = k_cache.shape
    _req(q, torch.bfloat16, "decode_attention.q")
    kv8 = _req_kv(k_cache, v_cache, "decode_attention")
    _req(slot, torch.int32, "decode_attention.slot")
    _req(seq_len, torch.int32, "decode_attention.seq_len")
    if Dk != D or D not in (64, 128) or Hq % Hkv or (Hq // Hkv) not in (1, 2, 3, 4, 6, 8) or v_cache.shape != k_cache.shape:
        raise HipOpsError(f"decode_attention: unsupported shape q={tuple(q.shape)} kv={tuple(k_cache.shape)}")
    if slot.numel() != B or seq_len.numel() != B:
        raise HipOpsError("decode_attention: slot/seq_len must have B entries")
    if chunk <= 0:
        raise HipOpsError("decode_attention: chunk must be positive")
    max_splits = decode_splits(MAXS, chunk)
    splits = max_splits if splits is None else int(splits)
    if not 1 <= splits <= max_splits:
        raise HipOpsError(f"decode_attention: splits {splits} outside [1, {max_splits}]")
    ps_max = 0
    pk = pv = plen = prows = None
    if prefix is not None:
        # the shared prefix on the MFMA prefill kernel in prefix mode: K / V
        # rows of the prefix slot, ps_max key splits per query tile
        pk, pv, plen = prefix.k, prefix.v, prefix.length
        _req(pk, k_cache.dtype, "decode_attention.prefix.k")
        _req(pv, k_cache.dtype, "decode_attention.prefix.v")
        _req(plen, torch.int32, "decode_attention.prefix.length")
        if tuple(pk.shape) != (Hkv, MAXS, D) or tuple(pv.shape) != (Hkv, MAXS, D) or plen.numel() != 1:
            raise HipOpsError(f"decode_attention: prefix k {tuple(pk.shape)} / v {tuple(pv.shape)} do not match "
                              f"kv {tuple(k_cache.shape)}")
        ps_max = prefix_mfma_splits(B, Hq // Hkv, Hkv)
        prows = getattr(prefix, "rows", None)
        if prows is not None:
            _req(prows, torch.int32, "decode_attention.prefix.rows")
            if prows.numel() < B:
                raise HipOpsError("decode_attention: prefix.rows has fewer than B entries")
        if workspace is not None and workspace[1].numel() < 2 * B * Hq * (splits + ps_max):
            raise HipOpsError(f"decode_attention: workspace holds fewer than {splits} + {ps_max} partials per row")
    if fork is not None:
        _req(fork, torch.int32, "decode_attention.fork")
        if fork.numel() < 2 * S or not fork.is_contiguous():
            raise HipOpsError(f"decode_attention: fork table must be a contiguous int32 [{S}, 2]")
    out = torch.empty_like(q) if out is None else out
    _req_out(out, torch.bfloat16, B * Hq * D, "decode_attention.out")
    if splits > 1 or ps_max:
        if workspace is None:
            workspace = decode_workspace(B, Hq, Hkv, D, MAXS, q.device, chunk, ps_max)
        part_o, part_ml = workspace
        n = B * Hq * (splits + ps_max)
        if part_o.numel() < n * D or part_ml.numel() < n * 2:
            raise HipOpsError("decode_attention: workspace too small")
    else:
        part_o = part_ml = None
    _check(lib().dmcp_decode_attention(_ptr(q), _ptr(k_cache), _ptr(v_cache), _ptr(slot), _ptr(seq_len), _ptr(out),
                                       _ptr(part_o), _ptr(part_ml), B, Hq, Hkv, D, MAXS, S, chunk, splits,
                                       float(scale), _ptr(pk), _ptr(pv), _ptr(plen), ps_max, kv8, _ptr(prows),
                                       _ptr(fork), _stream()), "dmcp_decode_attention")
    return out


def prefill_supported(n_heads: int, n_kv_heads: int, head_dim: int) -> bool:
    """Shapes the MFMA prefill-attention kernel covers (any GQA group)."""
    return head_dim in (64, 128) and n_kv_heads > 0 and n_heads % n_kv_heads == 0


PREFILL_VARIANTS = {64: (0, 1), 128: (0, 1)}  # waves per block: 0 = 4, 1 = 8


def prefill_splits(T: int, Hq: int, Hkv: int, variant: int = 0, target_blocks: int = 1024) -> int:
    """Key splits per query tile so that a prefill launch has ~4 blocks per
    CU (1024 on 256 CUs): a 2,100-token class is only 33 x 8 = 264 tiles
    (measured: 177 -> 165 us with 2 splits, profiles/prefill_attn_r2.md)."""
    cols = 128 * (2 if variant == 1 else 1)
    blocks = -(-T * (Hq // Hkv) // cols) * Hkv
    return max(1, min(8, -(-target_blocks // max(1, blocks))))


def prefill_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, slot: int, start: int,
                      prefix_slot: Optional[int] = None, prefix_len: int = 0, scale: float = 1.0,
                      out: Optional[torch.Tensor] = None, variant: int = 0, nsplit: int = 0) -> torch.Tensor:
    """Causal attention of q [T, Hq, D] (positions [start, start+T) of
    ``slot``, K/V already appended by rope_kv) over keys [0, start+T) of the
    caches [S, Hkv, MAXS, D]; keys [0, prefix_len) are read in place from
    ``prefix_slot`` (the shared prefix, no per-sequence copy).  One MFMA
    kernel (csrc/prefill_attn.hip); ``nsplit`` > 1 splits every query tile's
    keys over that many blocks plus a merge kernel (0 = :func:`prefill_splits`).
    Returns [T, Hq, D] bf16."""
    T, Hq, D = q.shape
    S, Hkv, MAXS, Dk = k_cache.shape
    _req(q, torch.bfloat16, "prefill_attention.q")
    kv8 = _req_kv(k_cache, v_cache, "prefill_attention")
    if Dk != D or v_cache.shape != k_cache.shape or not prefill_supported(Hq, Hkv, D):
        raise HipOpsError(f"prefill_attention: unsupported shape q={tuple(q.shape)} kv={tuple(k_cache.shape)}")
    slot, start, prefix_len = int(slot), int(start), int(prefix_len)
    if not 0 <= slot < S or start < 0 or T < 1 or start + T > MAXS:
        raise HipOpsError(f"prefill_attention: slot {slot} / positions [{start}, {start + T}) outside "
                          f"{S} slots x {MAXS} positions")
    if prefix_len:
        if prefix_slot is None or not 0 <= int(prefix_slot) < S or not 0 < prefix_len <= start:
            raise HipOpsError(f"prefill_attention: prefix of {prefix_len} keys in slot {prefix_slot} must precede "
                              f"start {start}")
        pk, pv = k_cache[int(prefix_slot)], v_cache[int(prefix_slot)]
    else:
        pk = pv = None
    nsplit = int(nsplit) or prefill_splits(T, Hq, Hkv, variant)
    if variant not in PREFILL_VARIANTS[D] or not 1 <= nsplit <= 64:
        raise HipOpsError(f"prefill_attention: variant {variant} / nsplit {nsplit} not available for D={D}")
    out = torch.empty_like(q) if out is None else out
    _req_out(out, torch.bfloat16, T * Hq * D, "prefill_attention.out")
    part_o = part_ml = None
    if nsplit > 1:
        part_o = torch.empty(nsplit * T * Hq * D, dtype=torch.float32, device=q.device)
        part_ml = torch.empty(nsplit * T * Hq * 2, dtype=torch.float32, device=q.device)
    _check(lib().dmcp_prefill_attention(_ptr(q), _ptr(k_cache[slot]), _ptr(v_cache[slot]), _ptr(pk), _ptr(pv),
                                        _ptr(out), _ptr(part_o), _ptr(part_ml), T, start, prefix_len, Hq, Hkv, D,
                                        MAXS, float(scale), int(variant), int(nsplit), kv8, _stream()),
           "dmcp_prefill_attention")
    return out


VARLEN_COLS = 128  # query columns (token x q head of a kv group) per varlen work item: 4 waves x 32


_VARLEN_META: dict = {}  # the last prefill's work list: key -> (items, device int32 meta)


def _varlen_meta(key: tuple, device) -> tuple:
    """The varlen kernel's work list: items (sequence, 128-column tile) by
    descending key count (ties: sequence, then tile order), then the
    sequences' (row offset, length, start, slot, prefix length).  Validates
    every sequence."""
    offsets, slots, starts, prefix_slot, plens, G, S, MAXS, _ = key
    n = len(slots)
    off = np.asarray(offsets, dtype=np.int64)
    T = off[1:] - off[:-1]
    st = np.asarray(starts, dtype=np.int64)
    sl = np.asarray(slots, dtype=np.int64)
    P = np.asarray(plens, dtype=np.int64)
    bad = np.flatnonzero((T < 1) | (sl < 0) | (sl >= S) | (st < 0) | (st + T > MAXS))
    if bad.size:
        i = int(bad[0])
        raise HipOpsError(f"prefill_attention_varlen: sequence {i} (slot {int(sl[i])}, [{int(st[i])}, "
                          f"{int(st[i] + T[i])})) does not fit {S} slots x {MAXS} positions")
    ps_bad = prefix_slot is None or not 0 <= prefix_slot < S
    bad = np.flatnonzero((P != 0) & (ps_bad | (P < 0) | (P > st)))
    if bad.size:
        i = int(bad[0])
        raise HipOpsError(f"prefill_attention_varlen: prefix of {int(P[i])} keys in slot {prefix_slot} must precede "
                          f"start {int(st[i])}")
    ntile = -(-T * G // VARLEN_COLS)
    seq_of = np.repeat(np.arange(n, dtype=np.int64), ntile)
    ct = np.arange(int(ntile.sum()), dtype=np.int64) - np.repeat(np.cumsum(ntile) - ntile, ntile)
    last_tok = np.minimum(T[seq_of], ((ct + 1) * VARLEN_COLS + G - 1) // G)
    order = np.argsort(-(st[seq_of] + last_tok), kind="stable")
    items = np.stack([seq_of[order], ct[order]], 1).ravel()
    seqs = np.stack([off[:-1], T, st, sl, P], 1).ravel()
    meta = torch.from_numpy(np.concatenate([items, seqs]).astype(np.int32))
    if torch.device(device).type == "cuda":
        meta = meta.pin_memory()
    return len(order), meta.to(device, non_blocking=True)


def prefill_attention_varlen(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, offsets, slots, starts,
                             prefix_slot: Optional[int] = None, prefix_lens=None, scale: float = 1.0,
                             out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Packed multi-sequence prefill attention in ONE launch
    (csrc/prefill_attn.hip::prefill_varlen_kernel): q [Ttot, Hq, D], sequence
    i = rows [offsets[i], offsets[i+1]) at positions [starts[i], ...) of
    ``slots[i]``, its first ``prefix_lens[i]`` keys read in place from
    ``prefix_slot``.  Work items (sequence, 128-column tile) are ordered by
    descending key count on the host.  Returns [Ttot, Hq, D] bf16."""
    Ttot, Hq, D = q.shape
    S, Hkv, MAXS, Dk = k_cache.shape
    _req(q, torch.bfloat16, "prefill_attention_varlen.q")
    kv8 = _req_kv(k_cache, v_cache, "prefill_attention_varlen")
    if Dk != D or v_cache.shape != k_cache.shape or not prefill_supported(Hq, Hkv, D):
        raise HipOpsError(f"prefill_attention_varlen: unsupported shape q={tuple(q.shape)} kv={tuple(k_cache.shape)}")
    n = len(slots)
    if len(offsets) != n + 1 or len(starts) != n or int(offsets[0]) != 0 or int(offsets[-1]) != Ttot:
        raise HipOpsError("prefill_attention_varlen: offsets must run from 0 to Ttot with one entry per sequence + 1")
    G = Hq // Hkv
    plens = [int(x) for x in prefix_lens] if prefix_lens is not None else [0] * n
    key = (tuple(int(x) for x in offsets), tuple(int(x) for x in slots), tuple(int(x) for x in starts),
           None if prefix_slot is None else int(prefix_slot), tuple(plens), G, S, MAXS, str(q.device))
    hit = _VARLEN_META.get(key)
    if hit is None:
        # every layer of a batched prefill launches with the same sequences:
        # the work list is built (and copied to the device) once per prefill,
        # not per layer (16 x ~0.5-0.9 ms of host time per admission)
        hit = _varlen_meta(key, q.device)
        _VARLEN_META.clear()
        _VARLEN_META[key] = hit
    n_items, meta = hit
    out = torch.empty_like(q) if out is None else out
    _req_out(out, torch.bfloat16, Ttot * Hq * D, "prefill_attention_varlen.out")
    it_t, seq_t = meta[:2 * n_items], meta[2 * n_items:]
    if any(plens):
        pk, pv = k_cache[int(prefix_slot)], v_cache[int(prefix_slot)]
    else:
        pk = pv = None
    _check(lib().dmcp_prefill_varlen(_ptr(q), _ptr(k_cache), _ptr(v_cache), _ptr(pk), _ptr(pv), _ptr(out),
                                     _ptr(it_t), _ptr(seq_t), n_items, Hq, Hkv, D, MAXS, Hkv * MAXS * D,
                                     float(scale), kv8, _stream()), "dmcp_prefill_varlen")
    return out


PREFIX_MFMA_MAX_SPLITS = 16


def prefix_mfma_splits(rows: int, G: int, Hkv: int, target_blocks: int = 640) -> int:
    """Key splits of the decode step's shared prefix: ~2.5 blocks per CU over
    (128-column query tiles x kv heads x splits), at most 16 (the combine
    reads every split's partial; empty ones weigh 0).  Measured on the fp8
    step with a 4,151-token prefix (profiles/prefix_splits_r3.txt): 8
    splits at 320 rows (4.86 vs 5.35 ms for the former 256-key chunk
    kernel), 12-16 at 78 rows (parity).  ``DMCP_PREFIX_SPLITS`` overrides."""
    env = os.environ.get("DMCP_PREFIX_SPLITS")
    if env:
        return max(1, min(PREFIX_MFMA_MAX_SPLITS, int(env)))
    tiles = -(-rows * G // 128) * Hkv
    return max(1, min(PREFIX_MFMA_MAX_SPLITS, round(target_blocks / max(1, tiles))))


def decode_workspace(rows: int, Hq: int, Hkv: int, D: int, max_seq: int, device, chunk: int = 256,
                     prefix_slots: int = 0) -> tuple:
    """Split-K scratch (fp32 partial outputs + running max/sum) for up to
    ``rows`` query rows, plus ``prefix_slots`` shared-prefix partials per row."""
    splits = decode_splits(max_seq, chunk) + prefix_slots
    n = rows * Hq * splits
    return (torch.empty(n * D, dtype=torch.float32, device=device),
            torch.empty(n * 2, dtype=torch.float32, device=device))


def silu_mul(gate_up: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    _req(gate_up, torch.bfloat16, "silu_mul.gate_up")
    T = gate_up.numel() // gate_up.shape[-1]
    I2 = gate_up.shape[-1]
    if I2 % 16:
        raise HipOpsError("silu_mul: intermediate size must be a multiple of 8")
    I = I2 // 2
    if out is None:
        out = torch.empty((*gate_up.shape[:-1], I), dtype=torch.bfloat16, device=gate_up.device)
    _req_out(out, torch.bfloat16, T * I, "silu_mul.out")
    _check(lib().dmcp_silu_mul(_ptr(gate_up), _ptr(out), T, I, _stream()), "dmcp_silu_mul")
    return out


def masked_argmax(logits: torch.Tensor, mask: Optional[torch.Tensor] = None, vocab: Optional[int] = None,
                  out: Optional[torch.Tensor] = None, mask_idx: Optional[torch.Tensor] = None) -> torch.Tensor:
    """logits [B, ld] bf16; mask int32 bitsets, ceil(V/32) words per row:
    [B, W] (row b -> mask b), or [M, W] with ``mask_idx`` int32 [B] choosing
    a mask row per logits row.  None = all tokens allowed."""
    _req(logits, torch.bfloat16, "masked_argmax.logits")
    B, ld = logits.shape
    V = vocab or ld
    W = (V + 31) // 32
    if V > ld:
        raise HipOpsError("masked_argmax: vocab larger than row")
    n_masks = 0
    if mask is not None:
        _req(mask, torch.int32, "masked_argmax.mask")
        if mask_idx is not None:
            _req(mask_idx, torch.int32, "masked_argmax.mask_idx")
            if mask.dim() != 2 or mask.shape[1] != W or mask.shape[0] < 1 or mask_idx.numel() != B:
                raise HipOpsError(f"masked_argmax: mask table {tuple(mask.shape)} / mask_idx {mask_idx.numel()} "
                                  f"do not match B={B}, W={W}")
            n_masks = mask.shape[0]
        elif mask.shape != (B, W):
            raise HipOpsError(f"masked_argmax: mask shape {tuple(mask.shape)} != {(B, W)}")
    elif mask_idx is not None:
        raise HipOpsError("masked_argmax: mask_idx given without a mask table")
    out = torch.empty((B,), dtype=torch.int32, device=logits.device) if out is None else out
    _req_out(out, torch.int32, B, "masked_argmax.out")
    _check(lib().dmcp_masked_argmax(_ptr(logits), _ptr(mask), _ptr(mask_idx if mask is not None else None), n_masks,
                                    _ptr(out), B, V, ld, _stream()), "dmcp_masked_argmax")
    return out


def pgemm_set_waves(waves: int) -> int:
    """Waves per block of the MX prefill GEMMs: 4 (one per SIMD, 128 x 128
    each) or 8 (two per SIMD, 128 x 64 each).  Returns the previous value."""
    if waves not in (4, 8):
        raise HipOpsError(f"pgemm_set_waves: 4 or 8, got {waves}")
    return int(lib().dmcp_pgemm_set_waves(int(waves)))


def pgemm_set_bk(bk: int) -> int:
    """K per LDS stage of the MX prefill GEMMs: 128 (the default: a 2-slot
    ring of 128-B image rows; 4-wave block, K % 128 == 0, else the 64-deep
    kernel runs) or 64 (a 4-stage ring of 64-B rows).  Returns the previous
    value."""
    if bk not in (64, 128):
        raise HipOpsError(f"pgemm_set_bk: 64 or 128, got {bk}")
    return int(lib().dmcp_pgemm_set_bk(int(bk)))


def wgemm_set_aux(aux: int) -> int:
    """Cache policy of the weight-streaming GEMM's weight loads: 0 (default)
    or 2 (nt).  Returns the previous value."""
    if aux not in (0, 2):
        raise HipOpsError(f"wgemm_set_aux: 0 or 2, got {aux}")
    return int(lib().dmcp_wgemm_set_aux(int(aux)))


def pgemm_set_areg(on: int) -> int:
    """1: the MX prefill GEMM's 128-deep stages take the activation (A)
    operand through registers (global loads, ds_write_b128 into the same LDS
    image) and only the weights by LDS-DMA; 0 (default): both by LDS-DMA.
    Returns the previous value."""
    if on not in (0, 1):
        raise HipOpsError(f"pgemm_set_areg: 0 or 1, got {on}")
    return int(lib().dmcp_pgemm_set_areg(int(on)))


def pgemm_set_group(g: int) -> int:
    """M tiles per block-order group of the MX prefill GEMMs (the blocks of a
    group's N column run back to back on one XCD).  Returns the previous value."""
    if not 1 <= g <= 64:
        raise HipOpsError(f"pgemm_set_group: 1..64, got {g}")
    return int(lib().dmcp_pgemm_set_group(int(g)))


def kv_fork(k_cache: torch.Tensor, v_cache: torch.Tensor, src: int, dsts, start: int, end: int) -> None:
    """Slot ``src``'s K/V at positions [start, end) of every layer into each
    slot of ``dsts`` (<= 32): one launch for both caches
    ([layers, slots, Hkv, max_seq, D] bf16, or e4m3 bytes)."""
    _req_kv(k_cache, v_cache, "kv_fork")
    if k_cache.dim() != 5 or not k_cache.is_contiguous() or not v_cache.is_contiguous():
        raise HipOpsError("kv_fork: caches must be contiguous [layers, slots, Hkv, max_seq, D]")
    L, S, H, T, D = k_cache.shape
    dl = [int(d) for d in dsts]
    if not dl or end <= start:
        return
    if len(dl) > 32:
        for i in range(0, len(dl), 32):
            kv_fork(k_cache, v_cache, src, dl[i:i + 32], start, end)
        return
    arr = (ctypes.c_int32 * len(dl))(*dl)
    _check(lib().dmcp_kv_fork(_ptr(k_cache), _ptr(v_cache), L, S, H, T, D * k_cache.element_size(), int(src),
                              ctypes.cast(arr, ctypes.c_void_p),
                              len(dl), int(start), int(end), _stream()), "dmcp_kv_fork")


def embedding(table: torch.Tensor, ids: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    _req(table, torch.bfloat16, "embedding.table")
    _req(ids, torch.int32, "embedding.ids")
    V, H = table.shape
    if H % 8:
        raise HipOpsError("embedding: hidden size must be a multiple of 8")
    T = ids.numel()
    out = torch.empty((T, H), dtype=torch.bfloat16, device=table.device) if out is None else out
    _req_out(out, torch.bfloat16, T * H, "embedding.out")
    _check(lib().dmcp_embedding(_ptr(table), _ptr(ids), _ptr(out), T, H, V, _stream()), "dmcp_embedding")
    return out


def decode_embed_norm(table: torch.Tensor, tokens: torch.Tensor, positions: torch.Tensor,
                      weight: Optional[torch.Tensor], eps: float, src: Optional[torch.Tensor] = None,
                      last_ids: Optional[torch.Tensor] = None, mask_idx: Optional[torch.Tensor] = None,
                      mask_alt: Optional[torch.Tensor] = None, alt_token: int = -1) -> tuple:
    """Decode-step inputs in one launch: row r's token is
    ``last_ids[src[r]]`` where ``src[r] >= 0`` (else ``tokens[r]``); returns
    (resid = its embedding row, h = RMSNorm(resid) * weight -- None when
    ``weight`` is None --, seq_len = positions + 1).  With ``mask_alt``: a
    gathered token equal to ``alt_token`` sets ``mask_idx[r] = mask_alt[r]``
    where that is >= 0 (in place; the step's masked argmax reads it after).
    Capturable."""
    _req(table, torch.bfloat16, "decode_embed_norm.table")
    _req(tokens, torch.int32, "decode_embed_norm.tokens")
    _req(positions, torch.int32, "decode_embed_norm.positions")
    V, H = table.shape
    B = tokens.numel()
    if H % 8 or H > 8192:
        raise HipOpsError(f"decode_embed_norm: unsupported hidden size {H}")
    if positions.numel() != B:
        raise HipOpsError("decode_embed_norm: tokens / positions length mismatch")
    if weight is not None:
        _req(weight, torch.bfloat16, "decode_embed_norm.weight")
        if weight.numel() != H:
            raise HipOpsError("decode_embed_norm: weight size != hidden")
    if (src is None) != (last_ids is None):
        raise HipOpsError("decode_embed_norm: src and last_ids go together")
    if src is not None:
        _req(src, torch.int32, "decode_embed_norm.src")
        _req(last_ids, torch.int32, "decode_embed_norm.last_ids")
        if src.numel() != B or last_ids.numel() == 0:
            raise HipOpsError("decode_embed_norm: src length / last_ids size")
    if mask_alt is not None:
        _req(mask_alt, torch.int32, "decode_embed_norm.mask_alt")
        if mask_idx is None or src is None:
            raise HipOpsError("decode_embed_norm: mask_alt needs mask_idx and src")
        _req(mask_idx, torch.int32, "decode_embed_norm.mask_idx")
        if mask_alt.numel() != B or mask_idx.numel() != B:
            raise HipOpsError("decode_embed_norm: mask_idx / mask_alt length != rows")
    resid = torch.empty((B, H), dtype=torch.bfloat16, device=table.device)
    h = torch.empty_like(resid) if weight is not None else None
    seq_len = torch.empty(B, dtype=torch.int32, device=table.device)
    alt = mask_alt is not None
    _check(lib().dmcp_decode_embed_norm(_ptr(table), _ptr(tokens), _ptr(src), _ptr(last_ids), _ptr(positions),
                                        _ptr(weight), _ptr(resid), _ptr(h), _ptr(seq_len), B, H, V,
                                        0 if last_ids is None else last_ids.numel(), float(eps),
                                        _ptr(mask_idx) if alt else None, _ptr(mask_alt) if alt else None,
                                        int(alt_token), _stream()),
           "dmcp_decode_embed_norm")
    return resid, h, seq_len


# ------------------------------------------------------------------ fused GEMMs
FUSED_EPI = {"rope_kv": 0, "swiglu": 1, "resid": 2, "bf16": 3}
FUSED_MAX_ROWS = 128  # dmcp_fused_gemm_max_rows()


def _fused_xw(x: torch.Tensor, w: torch.Tensor, name: str) -> tuple:
    _req(x, torch.bfloat16, f"{name}.x")
    _req(w, torch.bfloat16, f"{name}.w")
    if x.dim() != 2 or w.dim() != 2 or x.shape[1] != w.shape[1]:
        raise HipOpsError(f"{name}: x {tuple(x.shape)} / w {tuple(w.shape)} are not [M, K] / [N, K]")
    M, K = x.shape
    if not 1 <= M <= FUSED_MAX_ROWS or K % 32:
        raise HipOpsError(f"{name}: needs 1 <= M <= {FUSED_MAX_ROWS} rows and K % 32 == 0 (M={M}, K={K})")
    return M, K, w.shape[0]


def _fused(epi: str, wk: int, x, w, out, M, K, N, eps=0.0, inter=0, pos=None, slot=None, cos_sin=None,
           q_out=None, k_cache=None, v_cache=None, Hq=0, Hkv=0, D=0, max_seq=0, max_pos=0, num_slots=0,
           kv8=0) -> None:
    if wk not in (4, 8, 16):
        raise HipOpsError(f"fused_gemm: wk must be 4, 8 or 16 (got {wk})")
    _check(lib().dmcp_fused_gemm(FUSED_EPI[epi], wk, _ptr(x), _ptr(w), _ptr(out), M, K, N, float(eps), inter,
                                 _ptr(pos), _ptr(slot), _ptr(cos_sin), _ptr(q_out), _ptr(k_cache), _ptr(v_cache),
                                 Hq, Hkv, D, max_seq, max_pos, num_slots, kv8, _stream()), f"dmcp_fused_gemm[{epi}]")


def fused_rope_kv(x: torch.Tensor, w: torch.Tensor, eps: float, pos: torch.Tensor, slot: torch.Tensor,
                  cos_sin: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, n_q_heads: int,
                  q_out: Optional[torch.Tensor] = None, wk: int = 8) -> torch.Tensor:
    """q = RoPE(rms(x) . w[:Hq*D]^T); RoPE(k) and v appended to the KV cache at
    (slot[m], :, pos[m]) -- the RMSNorm weight must be folded into ``w``.
    x [M, K]; w [(Hq + 2 Hkv) D, K]; caches [S, Hkv, MAXS, D].  Returns q [M, Hq, D]."""
    M, K, N = _fused_xw(x, w, "fused_rope_kv")
    S, Hkv, MAXS, D = k_cache.shape
    kv8 = _req_kv(k_cache, v_cache, "fused_rope_kv")
    _req(pos, torch.int32, "fused_rope_kv.pos")
    _req(slot, torch.int32, "fused_rope_kv.slot")
    _req(cos_sin, torch.float32, "fused_rope_kv.cos_sin")
    if (v_cache.shape != k_cache.shape or N != (n_q_heads + 2 * Hkv) * D or D % 32 or pos.numel() != M
            or slot.numel() != M or cos_sin.dim() != 3 or tuple(cos_sin.shape[1:]) != (D // 2, 2)):
        raise HipOpsError(f"fused_rope_kv: shape mismatch (w {tuple(w.shape)}, cache {tuple(k_cache.shape)}, "
                          f"Hq {n_q_heads}, cos_sin {tuple(cos_sin.shape)})")
    if q_out is None:
        q_out = torch.empty((M, n_q_heads, D), dtype=torch.bfloat16, device=x.device)
    _req_out(q_out, torch.bfloat16, M * n_q_heads * D, "fused_rope_kv.q_out")
    _fused("rope_kv", wk, x, w, None, M, K, N, eps, pos=pos, slot=slot, cos_sin=cos_sin, q_out=q_out,
           k_cache=k_cache, v_cache=v_cache, Hq=n_q_heads, Hkv=Hkv, D=D, max_seq=MAXS,
           max_pos=cos_sin.shape[0], num_slots=S, kv8=kv8)
    return q_out


def fused_swiglu(x: torch.Tensor, w: torch.Tensor, eps: float, out: Optional[torch.Tensor] = None,
                 wk: int = 4) -> torch.Tensor:
    """silu(rms(x) . w[:I]^T) * (rms(x) . w[I:]^T); w [2I, K] (norm weight folded in)."""
    M, K, N = _fused_xw(x, w, "fused_swiglu")
    if N % 32:
        raise HipOpsError(f"fused_swiglu: 2I = {N} must be a multiple of 32")
    inter = N // 2
    if out is None:
        out = torch.empty((M, inter), dtype=torch.bfloat16, device=x.device)
    _req_out(out, torch.bfloat16, M * inter, "fused_swiglu.out")
    _fused("swiglu", wk, x, w, out, M, K, N, eps, inter=inter)
    return out


def fused_resid(x: torch.Tensor, w: torch.Tensor, residual: torch.Tensor, wk: int = 8) -> torch.Tensor:
    """residual += x . w^T (in place, bf16); x [M, K], w [N, K], residual [M, N]."""
    M, K, N = _fused_xw(x, w, "fused_resid")
    if N % 16:
        raise HipOpsError(f"fused_resid: N = {N} must be a multiple of 16")
    _req(residual, torch.bfloat16, "fused_resid.residual")
    if tuple(residual.shape) != (M, N):
        raise HipOpsError(f"fused_resid: residual {tuple(residual.shape)} != {(M, N)}")
    _fused("resid", wk, x, w, residual, M, K, N)
    return residual


# Above 512 rows hipBLASLt's large tiles win: the decode step with the
# weight-streaming GEMMs vs hipBLASLt was 6.56 / 6.53 ms at 512 rows, 7.94 /
# 7.54 at 640, 9.13 / 8.79 at 768, 11.83 / 11.48 at 1,024 (kernel extended to
# 1,024 rows for that measurement: profiles/decode_step_512rows_r3.txt)
WGEMM_MAX_ROWS = 512


def wgemm_plan(M: int, N: int, K: int, swiglu: bool = False, target_blocks: int = 192) -> tuple:
    """(K slices S, M parts) of the weight-streaming GEMM (csrc/wgemm.hip).

    Below 384 rows (tuned at 78 and 320 rows, profiles/wgemm_r3.txt): M parts
    of <= 192 rows (<= 3 16-row tiles per wave), then K slices (powers of
    two, whole 64-deep chunks, >= 512 deep) until 64-row weight tiles x parts
    x slices covers ~3/4 of the 256 CUs; SwiGLU writes its output directly (S = 1)
    and splits M instead.

    From 384 rows a block holds ~100-150 KB of LDS, so one block per CU: a
    grid past 256 blocks runs a second, mostly idle wave (the 384-block SwiGLU
    at 448 rows made the whole step 11 % slower than hipBLASLt).  There the
    plan minimises waves x staged bytes per block ((weight rows + X rows
    staged, the part rounded to 32) x K / S, at the measured ~33 KB/us per CU) plus the split-K partials'
    round trip, over M parts of 256 / 192 / 128 rows."""
    tiles = (N // 2 if swiglu else N) // 64
    if M >= 384:
        nb = 128 if swiglu else 64
        best = None
        for mparts in sorted({-(-M // 256), -(-M // 192), -(-M // 128)}):
            rows = (-(-M // mparts) + 15) // 16 * 16
            mt = -(-rows // 64)
            if mt > 4:
                continue
            mr = -(-rows // 32) * 32  # X rows the kernel stages (the part rounded to 32)
            for S in ((1,) if swiglu else (1, 2, 4, 8)):
                if K % (64 * S):
                    continue
                blocks = tiles * mparts * S
                us = -(-blocks // 256) * (nb + mr) * 2 * (K / S) / 33e3 + (0 if swiglu else S * M * N * 8 / 5e6)
                key = (round(us, 3), -blocks)
                if best is None or key < best[0]:
                    best = (key, S, mparts)
        return best[1], best[2]
    mparts = max(1, -(-M // 192))
    if swiglu:
        while tiles * mparts < target_blocks and -(-M // (mparts + 1)) >= 16:
            mparts += 1
        return 1, mparts
    # K slices of >= 512 (the split sweep at 40-320 rows: O / QKV at K = 2,048
    # fastest with 4 slices, not 8 -- profiles/wgemm_split_sweep_r6.jsonl)
    S = 1
    while tiles * mparts * S < target_blocks and S < 8 and K % (64 * S * 2) == 0 and K // (S * 2) >= 512:
        S *= 2
    return S, mparts


def _wgemm_args(x: torch.Tensor, w: torch.Tensor, name: str) -> tuple:
    _req(x, torch.bfloat16, f"{name}.x")
    _req(w, torch.bfloat16, f"{name}.w")
    if x.dim() != 2 or w.dim() != 2 or x.shape[1] != w.shape[1]:
        raise HipOpsError(f"{name}: x {tuple(x.shape)} / w {tuple(w.shape)} are not [M, K] / [N, K]")
    M, K = x.shape
    N = w.shape[0]
    if not 1 <= M <= WGEMM_MAX_ROWS or K % 64 or N % 64:
        raise HipOpsError(f"{name}: needs 1 <= M <= {WGEMM_MAX_ROWS}, K % 64 == 0, N % 64 == 0 (M={M} K={K} N={N})")
    return M, K, N


def lm_head_supported(vocab: int, hidden: int) -> bool:
    """Shapes of the fused LM head + masked argmax (csrc/wgemm.hip MODE_ARGMAX)."""
    return vocab % 64 == 0 and hidden % 64 == 0


def lm_head_workspace(vocab: int, device, rows: int = WGEMM_MAX_ROWS) -> torch.Tensor:
    """(max, id) pairs of every 64-id vocabulary tile of ``rows`` rows (fp32 pairs)."""
    return torch.empty(2 * (vocab // 64) * rows, dtype=torch.float32, device=device)


def lm_head_argmax(x: torch.Tensor, w: torch.Tensor, masks: torch.Tensor, mask_idx: torch.Tensor,
                   out: Optional[torch.Tensor] = None, workspace: Optional[torch.Tensor] = None) -> torch.Tensor:
    """ids[m] = argmax over the vocabulary ids allowed by mask row
    ``mask_idx[m]`` of bf16(x[m] . w[v]) -- the LM head GEMM and the grammar-
    masked greedy selection in one weight-streaming kernel + a per-row
    reduction; the [M, V] logits are never written.  x [M, K] bf16 (any M:
    chunks of WGEMM_MAX_ROWS), w [V, K] bf16, masks int32 [n_masks, ceil(V/32)],
    mask_idx int32 [M].  Ties -> lowest id; nothing allowed -> 0 (as
    :func:`masked_argmax`).  Capturable."""
    _req(x, torch.bfloat16, "lm_head_argmax.x")
    _req(w, torch.bfloat16, "lm_head_argmax.w")
    _req(masks, torch.int32, "lm_head_argmax.masks")
    _req(mask_idx, torch.int32, "lm_head_argmax.mask_idx")
    M, K = x.shape
    V = w.shape[0]
    if w.shape[1] != K or not lm_head_supported(V, K):
        raise HipOpsError(f"lm_head_argmax: x {tuple(x.shape)} / w {tuple(w.shape)} (needs V % 64 == 0, K % 64 == 0)")
    W = (V + 31) // 32
    if masks.dim() != 2 or masks.shape[1] != W or mask_idx.numel() != M:
        raise HipOpsError(f"lm_head_argmax: masks {tuple(masks.shape)} / mask_idx {mask_idx.numel()} vs M={M}, W={W}")
    if out is None:
        out = torch.empty(M, dtype=torch.int32, device=x.device)
    _req_out(out, torch.int32, M, "lm_head_argmax.out")
    rows = min(M, WGEMM_MAX_ROWS)
    if workspace is None:
        workspace = lm_head_workspace(V, x.device, rows)
    if workspace.dtype != torch.float32 or workspace.numel() < 2 * (V // 64) * rows:
        raise HipOpsError("lm_head_argmax: workspace too small")
    for m0 in range(0, M, WGEMM_MAX_ROWS):
        mc = min(WGEMM_MAX_ROWS, M - m0)
        mparts = -(-mc // 256)  # the fewest parts: every weight tile is read once per part
        _check(lib().dmcp_lm_head_argmax(_ptr(x[m0:m0 + mc]), _ptr(w), _ptr(masks), _ptr(mask_idx[m0:m0 + mc]),
                                         masks.shape[0], W, _ptr(workspace), _ptr(out[m0:m0 + mc]), mc, V, K,
                                         mparts, _stream()), "dmcp_lm_head_argmax")
    return out


def _wgemm_ws(workspace: torch.Tensor, n: int, name: str) -> None:
    if workspace.dtype != torch.float32 or not workspace.is_contiguous() or workspace.numel() < n:
        raise HipOpsError(f"{name}: workspace needs {n} contiguous fp32 elements")


def wgemm(x: torch.Tensor, w: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """x . w^T in bf16 (F.linear) on the weight-streaming kernel; M <= WGEMM_MAX_ROWS."""
    M, K, N = _wgemm_args(x, w, "wgemm")
    _, mparts = wgemm_plan(M, N, K)
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=x.device)
    _req_out(out, torch.bfloat16, M * N, "wgemm.out")
    _check(lib().dmcp_wgemm(_ptr(x), _ptr(w), _ptr(out), None, M, N, K, 1, mparts, 0, 0, _stream()), "dmcp_wgemm")
    return out


def wgemm_swiglu(x: torch.Tensor, w: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """silu(x . w[:I]^T) * (x . w[I:]^T) -- the gate/up projection with SwiGLU
    in its epilogue (w = [gate; up], [2I, K], I % 64 == 0); returns [M, I]."""
    M, K, N = _wgemm_args(x, w, "wgemm_swiglu")
    if N % 128:
        raise HipOpsError(f"wgemm_swiglu: 2I = {N} must be a multiple of 128")
    inter = N // 2
    _, mparts = wgemm_plan(M, N, K, swiglu=True)
    if out is None:
        out = torch.empty((M, inter), dtype=torch.bfloat16, device=x.device)
    _req_out(out, torch.bfloat16, M * inter, "wgemm_swiglu.out")
    _check(lib().dmcp_wgemm(_ptr(x), _ptr(w), _ptr(out), None, M, N, K, 1, mparts, 2, inter, _stream()),
           "dmcp_wgemm[swiglu]")
    return out


def wgemm_partials(x: torch.Tensor, w: torch.Tensor, workspace: torch.Tensor, splits: int = 0) -> int:
    """fp32 split-K partials of x . w^T into ``workspace`` [S, M, N]; returns S."""
    M, K, N = _wgemm_args(x, w, "wgemm_partials")
    S, mparts = wgemm_plan(M, N, K)
    S = splits or S
    if K % (64 * S):
        raise HipOpsError(f"wgemm_partials: K={K} does not split into {S} slices of whole 64-deep chunks")
    _wgemm_ws(workspace, S * M * N, "wgemm_partials")
    _check(lib().dmcp_wgemm(_ptr(x), _ptr(w), None, _ptr(workspace), M, N, K, S, mparts, 1, 0, _stream()),
           "dmcp_wgemm[partials]")
    return S


def wgemm_resid_norm(x: torch.Tensor, w: torch.Tensor, residual: torch.Tensor, norm_w: torch.Tensor, eps: float,
                     workspace: torch.Tensor, out: Optional[torch.Tensor] = None, splits: int = 0) -> torch.Tensor:
    """residual += bf16(x . w^T) (in place); returns RMSNorm(residual) * norm_w
    -- F.linear + add_rmsnorm as one split-K GEMM + one reduction per row that
    adds the residual and normalises.  x [M, K] (M <= WGEMM_MAX_ROWS), w [N, K]."""
    M, K, N = _wgemm_args(x, w, "wgemm_resid_norm")
    _req(residual, torch.bfloat16, "wgemm_resid_norm.residual")
    _req(norm_w, torch.bfloat16, "wgemm_resid_norm.norm_w")
    if tuple(residual.shape) != (M, N) or norm_w.numel() != N or N > 8192:
        raise HipOpsError("wgemm_resid_norm: residual / norm weight shape mismatch")
    S, mparts = wgemm_plan(M, N, K)
    S = splits or S
    if K % (64 * S):
        raise HipOpsError(f"wgemm_resid_norm: K={K} does not split into {S} slices")
    _wgemm_ws(workspace, S * M * N, "wgemm_resid_norm")
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=x.device)
    _req_out(out, torch.bfloat16, M * N, "wgemm_resid_norm.out")
    _check(lib().dmcp_wgemm_resid_norm(_ptr(x), _ptr(w), _ptr(workspace), _ptr(residual), _ptr(norm_w), _ptr(out),
                                       M, K, N, S, mparts, float(eps), _stream()), "dmcp_wgemm_resid_norm")
    return out


def wgemm_rope_kv(x: torch.Tensor, w: torch.Tensor, pos: torch.Tensor, slot: torch.Tensor, cos_sin: torch.Tensor,
                  k_cache: torch.Tensor, v_cache: torch.Tensor, n_q_heads: int, workspace: torch.Tensor,
                  q_out: Optional[torch.Tensor] = None, splits: int = 0) -> torch.Tensor:
    """rope_kv(F.linear(x, w), ...) as one split-K GEMM + one reduction per row
    (RoPE, the q write and the K/V-cache append).  x [M, K] (M <= WGEMM_MAX_ROWS);
    returns q [M, Hq, D]."""
    M, K, N = _wgemm_args(x, w, "wgemm_rope_kv")
    S_, Hkv, MAXS, D = k_cache.shape
    kv8 = _req_kv(k_cache, v_cache, "wgemm_rope_kv")
    _req(pos, torch.int32, "wgemm_rope_kv.pos")
    _req(slot, torch.int32, "wgemm_rope_kv.slot")
    _req(cos_sin, torch.float32, "wgemm_rope_kv.cos_sin")
    if v_cache.shape != k_cache.shape or N != (n_q_heads + 2 * Hkv) * D or D % 16 or N > 8192:
        raise HipOpsError(f"wgemm_rope_kv: w {tuple(w.shape)} does not match Hq={n_q_heads} / kv {tuple(k_cache.shape)}")
    if pos.numel() != M or slot.numel() != M or cos_sin.dim() != 3 or tuple(cos_sin.shape[1:]) != (D // 2, 2):
        raise HipOpsError("wgemm_rope_kv: pos/slot/cos_sin shape mismatch")
    S, mparts = wgemm_plan(M, N, K)
    S = splits or S
    if K % (64 * S):
        raise HipOpsError(f"wgemm_rope_kv: K={K} does not split into {S} slices")
    _wgemm_ws(workspace, S * M * N, "wgemm_rope_kv")
    if q_out is None:
        q_out = torch.empty((M, n_q_heads, D), dtype=torch.bfloat16, device=x.device)
    _req_out(q_out, torch.bfloat16, M * n_q_heads * D, "wgemm_rope_kv.q_out")
    _check(lib().dmcp_wgemm_rope_kv(_ptr(x), _ptr(w), _ptr(workspace), _ptr(pos), _ptr(slot), _ptr(cos_sin),
                                    _ptr(q_out), _ptr(k_cache), _ptr(v_cache), M, K, n_q_heads, Hkv, D, MAXS,
                                    cos_sin.shape[0], S_, kv8, S, mparts, _stream()), "dmcp_wgemm_rope_kv")
    return q_out


def wgemm_workspace(rows: int, n_max: int, device) -> torch.Tensor:
    """Partials scratch for the split-K weight-streaming GEMMs of a step of up
    to ``rows`` rows and ``n_max`` output columns (at most 8 slices)."""
    return torch.empty(8 * rows * n_max, dtype=torch.float32, device=device)


def fused_linear_norm(x: torch.Tensor, w: torch.Tensor, eps: float, out: Optional[torch.Tensor] = None,
                      wk: int = 16) -> torch.Tensor:
    """rms(x) . w^T in bf16 (norm weight folded into w); the LM head."""
    M, K, N = _fused_xw(x, w, "fused_linear_norm")
    if N % 16:
        raise HipOpsError(f"fused_linear_norm: N = {N} must be a multiple of 16")
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=x.device)
    _req_out(out, torch.bfloat16, M * N, "fused_linear_norm.out")
    _fused("bf16", wk, x, w, out, M, K, N, eps)
    return out


# ---- MXFP8 prefill GEMMs (csrc/pgemm.hip) ----------------------------------
# A operand: MXFP8 activations (e4m3 bytes [M, K] + E8M0 exponents [M, K / 32]);
# B operand: e4m3 weights [N, K] + fp32 per-row scales [N]
# (dmcp.ops.reference.quantize_weight).  256 x 256 output tiles.
PGEMM_TILE_N = 256


def pgemm_supported(hidden: int, n_heads: int, n_kv_heads: int, head_dim: int, inter: int) -> bool:
    """Whether a model's four projections fit the MXFP8 prefill kernels."""
    return (head_dim == 64 and (n_heads + 2 * n_kv_heads) % 4 == 0 and hidden % 2048 == 0 and hidden <= 8192
            and (n_heads * head_dim) % 64 == 0 and inter % 128 == 0 and hidden % PGEMM_TILE_N == 0)


def _mx_args(aq: torch.Tensor, as_: torch.Tensor, name: str) -> tuple:
    _req(aq, torch.uint8, f"{name}.aq")
    _req(as_, torch.uint8, f"{name}.as")
    if aq.dim() != 2 or aq.shape[1] % 64 or tuple(as_.shape) != (aq.shape[0], aq.shape[1] // 32):
        raise HipOpsError(f"{name}: activations {tuple(aq.shape)} / scales {tuple(as_.shape)} are not "
                          f"[M, K] / [M, K/32] with K % 64 == 0")
    return aq.shape[0], aq.shape[1]


def _w8_args(wq: torch.Tensor, ws: torch.Tensor, K: int, name: str) -> int:
    _req(wq, torch.uint8, f"{name}.wq")
    _req(ws, torch.float32, f"{name}.ws")
    if wq.dim() != 2 or wq.shape[1] != K or ws.numel() != wq.shape[0]:
        raise HipOpsError(f"{name}: weight {tuple(wq.shape)} / scales {ws.numel()} vs K={K}")
    return wq.shape[0]


def mx_quant(x: torch.Tensor, q: Optional[torch.Tensor] = None, s: Optional[torch.Tensor] = None) -> tuple:
    """bf16 [M, K] -> MXFP8 (q [M, K] e4m3, s [M, K / 32] E8M0)."""
    _req(x, torch.bfloat16, "mx_quant.x")
    M, K = x.shape
    if K % 32:
        raise HipOpsError(f"mx_quant: K={K} is not a multiple of 32")
    q = torch.empty((M, K), dtype=torch.uint8, device=x.device) if q is None else q
    s = torch.empty((M, K // 32), dtype=torch.uint8, device=x.device) if s is None else s
    _req_out(q, torch.uint8, M * K, "mx_quant.q")
    _req_out(s, torch.uint8, M * K // 32, "mx_quant.s")
    _check(lib().dmcp_mx_quant(_ptr(x), _ptr(q), _ptr(s), M, K, _stream()), "dmcp_mx_quant")
    return q, s


def rmsnorm_mx(resid: torch.Tensor, weight: torch.Tensor, eps: float, add: Optional[torch.Tensor] = None,
               q: Optional[torch.Tensor] = None, s: Optional[torch.Tensor] = None) -> tuple:
    """resid += add (in place, when given); RMSNorm(resid) * weight -> MXFP8."""
    _req(resid, torch.bfloat16, "rmsnorm_mx.resid")
    _req(weight, torch.bfloat16, "rmsnorm_mx.weight")
    M, N = resid.shape
    if N % 2048 or N > 8192 or weight.numel() != N:
        raise HipOpsError(f"rmsnorm_mx: N={N} (needs N % 2048 == 0, N <= 8192, weight [N])")
    if add is not None:
        _req(add, torch.bfloat16, "rmsnorm_mx.add")
        if tuple(add.shape) != (M, N):
            raise HipOpsError(f"rmsnorm_mx: add {tuple(add.shape)} != {(M, N)}")
    q = torch.empty((M, N), dtype=torch.uint8, device=resid.device) if q is None else q
    s = torch.empty((M, N // 32), dtype=torch.uint8, device=resid.device) if s is None else s
    _req_out(q, torch.uint8, M * N, "rmsnorm_mx.q")
    _req_out(s, torch.uint8, M * N // 32, "rmsnorm_mx.s")
    _check(lib().dmcp_rmsnorm_mx(_ptr(resid), _ptr(add), _ptr(weight), _ptr(q), _ptr(s), M, N, float(eps),
                                 _stream()), "dmcp_rmsnorm_mx")
    return q, s


def pgemm(aq: torch.Tensor, as_: torch.Tensor, wq: torch.Tensor, ws: torch.Tensor,
          out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """bf16 [M, N] = A . W^T on the MX fp8 matrix cores (N % 256 == 0)."""
    M, K = _mx_args(aq, as_, "pgemm")
    N = _w8_args(wq, ws, K, "pgemm")
    if N % PGEMM_TILE_N:
        raise HipOpsError(f"pgemm: N={N} is not a multiple of {PGEMM_TILE_N}")
    out = torch.empty((M, N), dtype=torch.bfloat16, device=aq.device) if out is None else out
    _req_out(out, torch.bfloat16, M * N, "pgemm.out")
    _check(lib().dmcp_pgemm(_ptr(aq), _ptr(as_), _ptr(wq), _ptr(ws), _ptr(out), M, N, K, 0, _stream()), "dmcp_pgemm")
    return out


def pgemm_resid(aq: torch.Tensor, as_: torch.Tensor, wq: torch.Tensor, ws: torch.Tensor,
                resid: torch.Tensor) -> torch.Tensor:
    """resid [M, N] += bf16(A . W^T) (in place) -- the o / down projection."""
    M, K = _mx_args(aq, as_, "pgemm_resid")
    N = _w8_args(wq, ws, K, "pgemm_resid")
    _req(resid, torch.bfloat16, "pgemm_resid.resid")
    if N % PGEMM_TILE_N or tuple(resid.shape) != (M, N):
        raise HipOpsError(f"pgemm_resid: resid {tuple(resid.shape)} vs {(M, N)} (N % {PGEMM_TILE_N} == 0)")
    _check(lib().dmcp_pgemm(_ptr(aq), _ptr(as_), _ptr(wq), _ptr(ws), _ptr(resid), M, N, K, 1, _stream()),
           "dmcp_pgemm[resid]")
    return resid


def pgemm_swiglu(aq: torch.Tensor, as_: torch.Tensor, wq: torch.Tensor, ws: torch.Tensor,
                 q: Optional[torch.Tensor] = None, s: Optional[torch.Tensor] = None) -> tuple:
    """silu(A . Wg^T) * (A . Wu^T) as MXFP8 [M, I] (wq = [gate; up] [2I, K])."""
    M, K = _mx_args(aq, as_, "pgemm_swiglu")
    N = _w8_args(wq, ws, K, "pgemm_swiglu")
    inter = N // 2
    if N % 256:
        raise HipOpsError(f"pgemm_swiglu: 2I = {N} is not a multiple of 256")
    q = torch.empty((M, inter), dtype=torch.uint8, device=aq.device) if q is None else q
    s = torch.empty((M, inter // 32), dtype=torch.uint8, device=aq.device) if s is None else s
    _req_out(q, torch.uint8, M * inter, "pgemm_swiglu.q")
    _req_out(s, torch.uint8, M * inter // 32, "pgemm_swiglu.s")
    _check(lib().dmcp_pgemm_swiglu(_ptr(aq), _ptr(as_), _ptr(wq), _ptr(ws), _ptr(q), _ptr(s), M, inter, K,
                                   _stream()), "dmcp_pgemm_swiglu")
    return q, s


def pgemm_qkv(aq: torch.Tensor, as_: torch.Tensor, wq: torch.Tensor, ws: torch.Tensor, pos: torch.Tensor,
              slot: torch.Tensor, cos_sin: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
              n_q_heads: int, q_out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """rope_kv(A . W^T): q [M, Hq, 64] bf16 returned, k / v appended to the caches."""
    M, K = _mx_args(aq, as_, "pgemm_qkv")
    N = _w8_args(wq, ws, K, "pgemm_qkv")
    S_, Hkv, MAXS, D = k_cache.shape
    kv8 = _req_kv(k_cache, v_cache, "pgemm_qkv")
    _req(pos, torch.int32, "pgemm_qkv.pos")
    _req(slot, torch.int32, "pgemm_qkv.slot")
    _req(cos_sin, torch.float32, "pgemm_qkv.cos_sin")
    if D != 64 or N != (n_q_heads + 2 * Hkv) * D or N % PGEMM_TILE_N or v_cache.shape != k_cache.shape:
        raise HipOpsError(f"pgemm_qkv: w {tuple(wq.shape)} vs Hq={n_q_heads} / kv {tuple(k_cache.shape)} "
                          f"(head dim 64, N % {PGEMM_TILE_N} == 0)")
    if pos.numel() != M or slot.numel() != M or cos_sin.dim() != 3 or tuple(cos_sin.shape[1:]) != (D // 2, 2):
        raise HipOpsError("pgemm_qkv: pos/slot/cos_sin shape mismatch")
    q_out = torch.empty((M, n_q_heads, D), dtype=torch.bfloat16, device=aq.device) if q_out is None else q_out
    _req_out(q_out, torch.bfloat16, M * n_q_heads * D, "pgemm_qkv.q_out")
    _check(lib().dmcp_pgemm_qkv(_ptr(aq), _ptr(as_), _ptr(wq), _ptr(ws), _ptr(pos), _ptr(slot), _ptr(cos_sin),
                                _ptr(q_out), _ptr(k_cache), _ptr(v_cache), M, K, n_q_heads, Hkv, MAXS,
                                cos_sin.shape[0], S_, kv8, _stream()), "dmcp_pgemm_qkv")
    return q_out


def mx_probe(a: torch.Tensor, b: torch.Tensor, sa: torch.Tensor, sb: torch.Tensor) -> torch.Tensor:
    """One v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3 x e4m3) on raw lane fragments:
    a / b uint8 [64 lanes, 32], sa / sb int32 [64] (E8M0 in byte 0) -> the
    accumulator registers fp32 [64 lanes, 16].  The tests' layout check."""
    for t, n, shp in ((a, "a", (64, 32)), (b, "b", (64, 32))):
        _req(t, torch.uint8, f"mx_probe.{n}")
        if tuple(t.shape) != shp:
            raise HipOpsError(f"mx_probe.{n}: {tuple(t.shape)} != {shp}")
    for t, n in ((sa, "sa"), (sb, "sb")):
        _req(t, torch.int32, f"mx_probe.{n}")
        if t.numel() != 64:
            raise HipOpsError(f"mx_probe.{n}: needs 64 lanes")
    c = torch.empty((64, 16), dtype=torch.float32, device=a.device)
    _check(lib().dmcp_mx_probe(_ptr(a), _ptr(b), _ptr(sa), _ptr(sb), _ptr(c), _stream()), "dmcp_mx_probe")
    return c


# ---- decode GEMMs on MX fp8 (csrc/pgemm.hip wmx_kernel) ---------------------
# a 768-row step (the engine's max_rows at 512 slots) stays on the MX kernel:
# 3-6 M parts re-stream each weight tile from L2 instead of hipBLASLt's bf16
WMX_MAX_ROWS = 1024
def wmx_plan(M: int, N: int, K: int, swiglu: bool = False) -> tuple:
    """(K slices S, M parts) of the MX decode GEMM: parts of 256 or 128 staged
    rows, whichever stages fewer rows for M (each part re-streams its weight
    tile, an L2 hit on the same XCD); then the most power-of-two K slices
    (whole 64-deep stages, >= 256 deep) that keep the grid within one wave
    of blocks -- 256, or 512 when a 128-row part's ~50 KB of LDS lets two
    blocks share a CU.  SwiGLU (its output quantised in place) does not split K."""
    a, b = -(-M // 256), -(-M // 128)
    mparts = a if a * 256 <= b * 128 else b
    if swiglu:
        return 1, mparts
    cap = 512 if -(-M // mparts) <= 128 else 256
    blocks = (N // 64) * mparts
    S = 1
    while blocks * S * 2 <= cap and K % (64 * S * 2) == 0 and K // (S * 2) >= 256:
        S *= 2
    return S, mparts


def _wmx_args(xq, xs, wq, ws, name):
    M, K = _mx_args(xq, xs, name)
    N = _w8_args(wq, ws, K, name)
    if not 1 <= M <= WMX_MAX_ROWS or N % 64:
        raise HipOpsError(f"{name}: needs 1 <= M <= {WMX_MAX_ROWS}, N % 64 == 0 (M={M} N={N})")
    return M, K, N


def wgemm_mx_partials(xq: torch.Tensor, xs: torch.Tensor, wq: torch.Tensor, ws: torch.Tensor,
                      workspace: torch.Tensor, splits: int = 0) -> int:
    """fp32 split-K partials [S, M, N] of MXFP8 x . (e4m3 w * ws)^T; returns S."""
    M, K, N = _wmx_args(xq, xs, wq, ws, "wgemm_mx_partials")
    S, mparts = wmx_plan(M, N, K)
    S = splits or S
    if K % (64 * S):
        raise HipOpsError(f"wgemm_mx_partials: K={K} does not split into {S} slices")
    _wgemm_ws(workspace, S * M * N, "wgemm_mx_partials")
    _check(lib().dmcp_wgemm_mx(_ptr(xq), _ptr(xs), _ptr(wq), _ptr(ws), _ptr(workspace), None, None, M, N, K, S,
                               mparts, 1, 0, _stream()), "dmcp_wgemm_mx[partials]")
    return S


def wgemm_mx_swiglu(xq: torch.Tensor, xs: torch.Tensor, wq: torch.Tensor, ws: torch.Tensor,
                    q: Optional[torch.Tensor] = None, s: Optional[torch.Tensor] = None) -> tuple:
    """silu(gate) * up of the stacked e4m3 [gate; up] weight, as MXFP8 [M, I]."""
    M, K, N = _wmx_args(xq, xs, wq, ws, "wgemm_mx_swiglu")
    if N % 64:
        raise HipOpsError(f"wgemm_mx_swiglu: 2I = {N} must be a multiple of 64")
    inter = N // 2
    _, mparts = wmx_plan(M, N, K, swiglu=True)
    q = torch.empty((M, inter), dtype=torch.uint8, device=xq.device) if q is None else q
    s = torch.empty((M, inter // 32), dtype=torch.uint8, device=xq.device) if s is None else s
    _req_out(q, torch.uint8, M * inter, "wgemm_mx_swiglu.q")
    _req_out(s, torch.uint8, M * inter // 32, "wgemm_mx_swiglu.s")
    _check(lib().dmcp_wgemm_mx(_ptr(xq), _ptr(xs), _ptr(wq), _ptr(ws), None, _ptr(q), _ptr(s), M, N, K, 1, mparts, 2,
                               inter, _stream()), "dmcp_wgemm_mx[swiglu]")
    return q, s


def wgemm_mx_resid_norm(xq, xs, wq, ws, residual: torch.Tensor, norm_w: torch.Tensor, eps: float,
                        workspace: torch.Tensor, mx: bool = True, out: Optional[tuple] = None):
    """residual += bf16(x . w^T); returns RMSNorm(residual) * norm_w as MXFP8
    (q, s) -- or, ``mx=False``, as bf16 (the last layer: the LM head's input)."""
    M, K, N = _wmx_args(xq, xs, wq, ws, "wgemm_mx_resid_norm")
    _req(residual, torch.bfloat16, "wgemm_mx_resid_norm.residual")
    _req(norm_w, torch.bfloat16, "wgemm_mx_resid_norm.norm_w")
    if tuple(residual.shape) != (M, N) or norm_w.numel() != N or N % 2048 or N > 8192:
        raise HipOpsError("wgemm_mx_resid_norm: residual / norm weight shape mismatch (N % 2048 == 0, <= 8192)")
    S = wgemm_mx_partials(xq, xs, wq, ws, workspace)
    if not mx:
        h = torch.empty((M, N), dtype=torch.bfloat16, device=xq.device) if out is None else out
        _req_out(h, torch.bfloat16, M * N, "wgemm_mx_resid_norm.out")
        _check(lib().dmcp_reduce_resid_norm(_ptr(workspace), S, _ptr(residual), _ptr(norm_w), _ptr(h), M, N,
                                            float(eps), _stream()), "dmcp_reduce_resid_norm")
        return h
    q, s = out if out is not None else (torch.empty((M, N), dtype=torch.uint8, device=xq.device),
                                        torch.empty((M, N // 32), dtype=torch.uint8, device=xq.device))
    _req_out(q, torch.uint8, M * N, "wgemm_mx_resid_norm.q")
    _req_out(s, torch.uint8, M * N // 32, "wgemm_mx_resid_norm.s")
    _check(lib().dmcp_reduce_resid_norm_mx(_ptr(workspace), S, _ptr(residual), _ptr(norm_w), _ptr(q), _ptr(s), M, N,
                                           float(eps), _stream()), "dmcp_reduce_resid_norm_mx")
    return q, s


def wgemm_mx_rope_kv(xq, xs, wq, ws, pos: torch.Tensor, slot: torch.Tensor, cos_sin: torch.Tensor,
                     k_cache: torch.Tensor, v_cache: torch.Tensor, n_q_heads: int, workspace: torch.Tensor,
                     q_out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """rope_kv(x . w^T) on the MX decode GEMM: q [M, Hq, D] returned, K/V appended."""
    M, K, N = _wmx_args(xq, xs, wq, ws, "wgemm_mx_rope_kv")
    S_, Hkv, MAXS, D = k_cache.shape
    kv8 = _req_kv(k_cache, v_cache, "wgemm_mx_rope_kv")
    _req(pos, torch.int32, "wgemm_mx_rope_kv.pos")
    _req(slot, torch.int32, "wgemm_mx_rope_kv.slot")
    _req(cos_sin, torch.float32, "wgemm_mx_rope_kv.cos_sin")
    if v_cache.shape != k_cache.shape or N != (n_q_heads + 2 * Hkv) * D or D % 16 or N > 8192:
        raise HipOpsError(f"wgemm_mx_rope_kv: w {tuple(wq.shape)} does not match Hq={n_q_heads} / kv "
                          f"{tuple(k_cache.shape)}")
    if pos.numel() != M or slot.numel() != M or cos_sin.dim() != 3 or tuple(cos_sin.shape[1:]) != (D // 2, 2):
        raise HipOpsError("wgemm_mx_rope_kv: pos/slot/cos_sin shape mismatch")
    S = wgemm_mx_partials(xq, xs, wq, ws, workspace)
    q_out = torch.empty((M, n_q_heads, D), dtype=torch.bfloat16, device=xq.device) if q_out is None else q_out
    _req_out(q_out, torch.bfloat16, M * n_q_heads * D, "wgemm_mx_rope_kv.q_out")
    _check(lib().dmcp_reduce_rope_kv(_ptr(workspace), S, _ptr(pos), _ptr(slot), _ptr(cos_sin), _ptr(q_out),
                                     _ptr(k_cache), _ptr(v_cache), M, n_q_heads, Hkv, D, MAXS, cos_sin.shape[0], S_,
                                     kv8, _stream()), "dmcp_reduce_rope_kv")
    return q_out


# ---------------------------------------------------------------- tgemm
# Steps of more than WGEMM_MAX_ROWS rows (up to the engine's max_rows) run on
# the large-tile GEMM (csrc/tgemm.hip): 256 weight rows x up to 256 rows per
# block, with the same fused consumers as the weight-streaming kernel.
TGEMM_MAX_ROWS = 1024
TGEMM_NB = 256


TGEMM_KC = 64  # K per LDS stage of the kernel (split-K slices are whole stages)


def tgemm_supported(N: int, K: int, swiglu: bool = False) -> bool:
    """The kernel's host contract (csrc/tgemm.hip dmcp_tgemm): K % 64, N % 256;
    SwiGLU (N = 2 I) needs I % 128, i.e. the same N % 256 -- one predicate
    with :func:`dmcp.models.llm.tgemm_shapes_ok` (tests/test_launch_plans.py)."""
    return K % TGEMM_KC == 0 and N > 0 and N % TGEMM_NB == 0


def tgemm_plan(M: int, N: int, K: int, mode: str = "part", cus: int = 256) -> tuple:
    """(K slices S, M parts) of the large-tile GEMM.  M parts of <= 256 rows
    (a part is staged rounded up to 64 rows); the plan minimises a time model
    fitted to the fused ops' (GEMM + reduction) measured (S, parts) sweeps at
    520-1,024 rows (profiles/tgemm_fused_sweep_r5.jsonl; mean error 10 %, the
    chosen plans within 0.7 us of the best over 12 shape x row cases): waves
    of blocks x max(MFMA time x 1.5, staged bytes at ~60 KB/us per CU) + 5 us +
    0.5 us per MB of fp32 split-K partials (written here, read back by the
    fused reduction).  ``mode``: "part" (fp32 partials, any S), "bf16",
    "swiglu" and "argmax" (S = 1)."""
    tiles = N // TGEMM_NB
    chunks = K // TGEMM_KC
    if mode == "argmax":  # measured best at 256-1,024 rows: the fewest parts
        return 1, -(-M // 256)
    if mode == "swiglu":  # measured best at 520-1,024 rows: 4 parts (64 x 4 = 256 blocks: one wave; 520 and 610
        return 1, max(-(-M // 256), 4)  # rows then stage 144 / 160 rows: a 3-stage ring, profiles/tgemm_xt_sweep_r6.jsonl)
    best = None
    for mparts in sorted({-(-M // r) for r in (256, 192, 160, 128, 96, 64)}):
        rows = (-(-M // mparts) + 15) // 16 * 16
        if rows > 256:
            continue
        xt = max(2, -(-rows // 32))  # staged X rows: 32 xt (the kernel's 32-row steps)
        for S in ((1,) if mode != "part" else range(1, 17)):
            cps = -(-chunks // S)
            if S > chunks or (S - 1) * cps >= chunks:
                continue
            blocks = tiles * mparts * S
            mfma_us = 1.5 * cps * 2 * 4 * xt * 2 * 16 / 2100.0  # 2 waves x 4 x XT x 2 k steps of 16 cycles per SIMD
            dma_us = cps * (TGEMM_NB + 32 * xt) * 2 * TGEMM_KC / 60e3
            us = -(-blocks // cus) * max(mfma_us, dma_us) + 5.0
            if mode == "part":
                us += S * M * N * 4 * 0.5e-6
            key = (round(us, 2), -blocks)
            if best is None or key < best[0]:
                best = (key, S, mparts)
    if best is None:
        raise HipOpsError(f"tgemm_plan: no plan for M={M} N={N} K={K}")
    return best[1], best[2]


def _tgemm_args(x: torch.Tensor, w: torch.Tensor, name: str, swiglu: bool = False) -> tuple:
    _req(x, torch.bfloat16, f"{name}.x")
    _req(w, torch.bfloat16, f"{name}.w")
    if x.dim() != 2 or w.dim() != 2 or x.shape[1] != w.shape[1]:
        raise HipOpsError(f"{name}: x {tuple(x.shape)} / w {tuple(w.shape)} are not [M, K] / [N, K]")
    M, K = x.shape
    N = w.shape[0]
    if not 1 <= M <= TGEMM_MAX_ROWS or not tgemm_supported(N, K, swiglu):
        raise HipOpsError(f"{name}: needs 1 <= M <= {TGEMM_MAX_ROWS}, K % {TGEMM_KC} == 0, N % {TGEMM_NB} == 0 "
                          f"(M={M} K={K} N={N})")
    return M, K, N


def _tg(x, w, y, part, M, N, K, S, mparts, mode, inter=0, masks=None, midx=None, n_masks=0, wwords=0, ids=None,
        name="dmcp_tgemm") -> None:
    _check(lib().dmcp_tgemm(_ptr(x), _ptr(w), _ptr(y), _ptr(part), M, N, K, S, mparts, mode, inter, _ptr(masks),
                            _ptr(midx), n_masks, wwords, _ptr(ids), _stream()), name)


def tgemm(x: torch.Tensor, w: torch.Tensor, out: Optional[torch.Tensor] = None, mparts: int = 0) -> torch.Tensor:
    """x . w^T in bf16 (F.linear) on the large-tile kernel; M <= TGEMM_MAX_ROWS."""
    M, K, N = _tgemm_args(x, w, "tgemm")
    mparts = mparts or tgemm_plan(M, N, K, "bf16")[1]
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=x.device)
    _req_out(out, torch.bfloat16, M * N, "tgemm.out")
    _tg(x, w, out, None, M, N, K, 1, mparts, 0)
    return out


def tgemm_swiglu(x: torch.Tensor, w: torch.Tensor, out: Optional[torch.Tensor] = None,
                 mparts: int = 0) -> torch.Tensor:
    """silu(x . w[:I]^T) * (x . w[I:]^T) on the large-tile kernel (w = [gate; up],
    I % 128 == 0); returns [M, I]."""
    M, K, N = _tgemm_args(x, w, "tgemm_swiglu", swiglu=True)
    inter = N // 2
    mparts = mparts or tgemm_plan(M, N, K, "swiglu")[1]
    if out is None:
        out = torch.empty((M, inter), dtype=torch.bfloat16, device=x.device)
    _req_out(out, torch.bfloat16, M * inter, "tgemm_swiglu.out")
    _tg(x, w, out, None, M, N, K, 1, mparts, 2, inter, name="dmcp_tgemm[swiglu]")
    return out


def tgemm_partials(x: torch.Tensor, w: torch.Tensor, workspace: torch.Tensor, splits: int = 0,
                   mparts: int = 0) -> int:
    """fp32 split-K partials of x . w^T into ``workspace`` [S, M, N]; returns S."""
    M, K, N = _tgemm_args(x, w, "tgemm_partials")
    S, mp = tgemm_plan(M, N, K, "part")
    S, mparts = splits or S, mparts or mp
    chunks = K // TGEMM_KC
    if S > chunks or (S - 1) * -(-chunks // S) >= chunks:
        raise HipOpsError(f"tgemm_partials: K={K} does not split into {S} non-empty slices")
    _wgemm_ws(workspace, S * M * N, "tgemm_partials")
    _tg(x, w, None, workspace, M, N, K, S, mparts, 1, name="dmcp_tgemm[partials]")
    return S


def tgemm_resid_norm(x: torch.Tensor, w: torch.Tensor, residual: torch.Tensor, norm_w: torch.Tensor, eps: float,
                     workspace: torch.Tensor, out: Optional[torch.Tensor] = None, splits: int = 0) -> torch.Tensor:
    """residual += bf16(x . w^T) (in place); returns RMSNorm(residual) * norm_w
    -- the large-tile split-K GEMM + wgemm.hip's fused reduction."""
    M, K, N = _tgemm_args(x, w, "tgemm_resid_norm")
    _req(residual, torch.bfloat16, "tgemm_resid_norm.residual")
    _req(norm_w, torch.bfloat16, "tgemm_resid_norm.norm_w")
    if tuple(residual.shape) != (M, N) or norm_w.numel() != N or N > 8192:
        raise HipOpsError("tgemm_resid_norm: residual / norm weight shape mismatch")
    S = tgemm_partials(x, w, workspace, splits)
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=x.device)
    _req_out(out, torch.bfloat16, M * N, "tgemm_resid_norm.out")
    _check(lib().dmcp_reduce_resid_norm(_ptr(workspace), S, _ptr(residual), _ptr(norm_w), _ptr(out), M, N,
                                        float(eps), _stream()), "dmcp_reduce_resid_norm")
    return out


def tgemm_rope_kv(x: torch.Tensor, w: torch.Tensor, pos: torch.Tensor, slot: torch.Tensor, cos_sin: torch.Tensor,
                  k_cache: torch.Tensor, v_cache: torch.Tensor, n_q_heads: int, workspace: torch.Tensor,
                  q_out: Optional[torch.Tensor] = None, splits: int = 0) -> torch.Tensor:
    """rope_kv(F.linear(x, w), ...) as the large-tile split-K GEMM + the fused
    RoPE / q write / KV-append reduction; returns q [M, Hq, D]."""
    M, K, N = _tgemm_args(x, w, "tgemm_rope_kv")
    S_, Hkv, MAXS, D = k_cache.shape
    kv8 = _req_kv(k_cache, v_cache, "tgemm_rope_kv")
    _req(pos, torch.int32, "tgemm_rope_kv.pos")
    _req(slot, torch.int32, "tgemm_rope_kv.slot")
    _req(cos_sin, torch.float32, "tgemm_rope_kv.cos_sin")
    if v_cache.shape != k_cache.shape or N != (n_q_heads + 2 * Hkv) * D or D % 16 or N > 8192:
        raise HipOpsError(f"tgemm_rope_kv: w {tuple(w.shape)} does not match Hq={n_q_heads} / kv {tuple(k_cache.shape)}")
    if pos.numel() != M or slot.numel() != M or cos_sin.dim() != 3 or tuple(cos_sin.shape[1:]) != (D // 2, 2):
        raise HipOpsError("tgemm_rope_kv: pos/slot/cos_sin shape mismatch")
    S = tgemm_partials(x, w, workspace, splits)
    if q_out is None:
        q_out = torch.empty((M, n_q_heads, D), dtype=torch.bfloat16, device=x.device)
    _req_out(q_out, torch.bfloat16, M * n_q_heads * D, "tgemm_rope_kv.q_out")
    _check(lib().dmcp_reduce_rope_kv(_ptr(workspace), S, _ptr(pos), _ptr(slot), _ptr(cos_sin), _ptr(q_out),
                                     _ptr(k_cache), _ptr(v_cache), M, n_q_heads, Hkv, D, MAXS, cos_sin.shape[0], S_,
                                     kv8, _stream()), "dmcp_reduce_rope_kv")
    return q_out


def tgemm_lm_head_argmax(x: torch.Tensor, w: torch.Tensor, masks: torch.Tensor, mask_idx: torch.Tensor,
                         out: Optional[torch.Tensor] = None, workspace: Optional[torch.Tensor] = None,
                         mparts: int = 0) -> torch.Tensor:
    """:func:`lm_head_argmax` on the large-tile kernel (V % 256 == 0): 256
    vocabulary ids per block, one (max, id) pair per block and row."""
    M, K, V = _tgemm_args(x, w, "tgemm_lm_head_argmax")
    _req(masks, torch.int32, "tgemm_lm_head_argmax.masks")
    _req(mask_idx, torch.int32, "tgemm_lm_head_argmax.mask_idx")
    W = (V + 31) // 32
    if masks.dim() != 2 or masks.shape[1] != W or mask_idx.numel() != M:
        raise HipOpsError(f"tgemm_lm_head_argmax: masks {tuple(masks.shape)} / mask_idx {mask_idx.numel()} vs M={M}")
    if out is None:
        out = torch.empty(M, dtype=torch.int32, device=x.device)
    _req_out(out, torch.int32, M, "tgemm_lm_head_argmax.out")
    need = 2 * (V // 64) * M  # one (max, id) pair per 64-id quarter tile and row
    if workspace is None:
        workspace = torch.empty(need, dtype=torch.float32, device=x.device)
    if workspace.dtype != torch.float32 or workspace.numel() < need:
        raise HipOpsError("tgemm_lm_head_argmax: workspace too small")
    mparts = mparts or tgemm_plan(M, V, K, "argmax")[1]
    _tg(x, w, None, workspace, M, V, K, 1, mparts, 3, 0, masks, mask_idx, masks.shape[0], W, out,
        name="dmcp_tgemm[argmax]")
    return out
