#!/usr/bin/env python3
"""Per-kernel microbenchmarks of the gfx950 ops against HBM speed of light.

Each op is timed with HIP events over many launches (after warm-up) and
reported as achieved bytes/s next to the MI355X HBM3E peak (~8 TB/s), plus the
time of the equivalent eager PyTorch composition for comparison.  One JSON
line per case; run on the GPU box:

    python scripts/bench_kernels.py > gpurun_out/kernels.jsonl
"""
from __future__ import annotations

import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dmcp.ops import hip, reference  # noqa: E402

PEAK_BYTES = 8.0e12


def timed(fn, iters=50, warmup=3):
    """Device time per call: ``iters`` calls captured in one hipGraph and
    replayed, so host-side launch cost (Python wrapper, ctypes) is excluded --
    the same way the decode loop runs them."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(warmup):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(3):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / (3 * iters) * 1e-3


def report(name, secs, nbytes, eager_secs=None, **cfg):
    out = {"kernel": name, "us": round(secs * 1e6, 2), "GBps": round(nbytes / secs / 1e9, 1),
           "pct_hbm_peak": round(100 * nbytes / secs / PEAK_BYTES, 1), "config": cfg}
    if eager_secs is not None:
        out["eager_us"] = round(eager_secs * 1e6, 2)
        out["speedup_vs_eager"] = round(eager_secs / secs, 2)
    print(json.dumps(out), flush=True)


def bench_decode_attention(B, L, Hq=32, Hkv=8, D=64, max_seq=4096, chunk=256, eager=True):
    dev = "cuda"
    kc = torch.randn(B, Hkv, max_seq, D, device=dev).to(torch.bfloat16)
    vc = torch.randn(B, Hkv, max_seq, D, device=dev).to(torch.bfloat16)
    q = torch.randn(B, Hq, D, device=dev).to(torch.bfloat16)
    slot = torch.arange(B, dtype=torch.int32, device=dev)
    sl = torch.full((B,), L, dtype=torch.int32, device=dev)
    ws = hip.decode_workspace(B, Hq, Hkv, D, max_seq, dev, chunk)
    out = torch.empty_like(q)
    t = timed(lambda: hip.decode_attention(q, kc, vc, slot, sl, 1 / math.sqrt(D), workspace=ws, chunk=chunk,
                                           out=out))
    nbytes = 2 * B * Hkv * L * D * 2 + 2 * q.numel() * 2
    k4, v4 = kc[:, :, :L], vc[:, :, :L]

    def sdpa():
        torch.nn.functional.scaled_dot_product_attention(q[:, :, None], k4, v4, enable_gqa=True)
    report("decode_attention", t, nbytes, timed(sdpa) if eager else None, B=B, L=L, Hq=Hq, Hkv=Hkv, D=D,
           chunk=chunk)


def bench_prefix_attention(B, P, Ls, Hq=32, Hkv=8, D=64, max_seq=8192, chunk=256):
    """Shared-prefix decode step: every row = P shared keys + Ls own keys.
    Bytes counted = what must be read at least once (prefix once, own keys
    per row); 'rowwise_us' = the same step without the prefix kernel (every
    row streams all P + Ls keys itself)."""
    from dmcp.ops.reference import SharedPrefix
    dev = "cuda"
    S = B + 1
    kc = torch.randn(S, Hkv, max_seq, D, device=dev).to(torch.bfloat16)
    vc = torch.randn(S, Hkv, max_seq, D, device=dev).to(torch.bfloat16)
    q = torch.randn(B, Hq, D, device=dev).to(torch.bfloat16)
    slot = torch.arange(B, dtype=torch.int32, device=dev)
    sl = torch.full((B,), P + Ls, dtype=torch.int32, device=dev)
    plen = torch.tensor([P], dtype=torch.int32, device=dev)
    pre = SharedPrefix(kc[B], vc[B], plen)
    ws = hip.decode_workspace(B, Hq, Hkv, D, max_seq, dev, chunk, hip.PREFIX_MFMA_MAX_SPLITS)
    out = torch.empty_like(q)
    t = timed(lambda: hip.decode_attention(q, kc, vc, slot, sl, 1 / math.sqrt(D), workspace=ws, chunk=chunk,
                                           out=out, prefix=pre))
    rowwise = timed(lambda: hip.decode_attention(q, kc, vc, slot, sl, 1 / math.sqrt(D), workspace=ws, chunk=chunk,
                                                 out=out))
    nbytes = 2 * Hkv * D * 2 * (P + B * Ls) + 2 * q.numel() * 2
    out_rec = {"rowwise_us": round(rowwise * 1e6, 2), "speedup_vs_rowwise": round(rowwise / t, 2)}
    report("decode_attention_shared_prefix", t, nbytes, None, B=B, P=P, Ls=Ls, Hq=Hq, Hkv=Hkv, D=D, chunk=chunk,
           **out_rec)


def bench_rmsnorm(rows, H=2048):
    x = torch.randn(rows, H, device="cuda").to(torch.bfloat16)
    r = torch.randn(rows, H, device="cuda").to(torch.bfloat16)
    w = torch.randn(H, device="cuda").to(torch.bfloat16)
    out = torch.empty_like(x)
    t = timed(lambda: hip.add_rmsnorm(x, w, 1e-5, residual=r, out=out))

    def eager():
        h = x + r
        return (h.float() * torch.rsqrt(h.float().pow(2).mean(-1, keepdim=True) + 1e-5)).to(x.dtype) * w
    report("add_rmsnorm", t, 4 * rows * H * 2, timed(eager), rows=rows, H=H)


def bench_silu(rows, I=8192):
    gu = torch.randn(rows, 2 * I, device="cuda").to(torch.bfloat16)
    out = torch.empty(rows, I, device="cuda", dtype=torch.bfloat16)
    t = timed(lambda: hip.silu_mul(gu, out))
    report("silu_mul", t, 3 * rows * I * 2, timed(lambda: reference.silu_mul(gu)), rows=rows, I=I)


def bench_rope(T, Hq=32, Hkv=8, D=64, max_seq=4096):
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device="cuda").to(torch.bfloat16)
    kc = torch.zeros(T, Hkv, max_seq, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    cs = reference.rope_tables(max_seq, D, device="cuda")
    pos = torch.randint(0, max_seq, (T,), dtype=torch.int32, device="cuda")
    slot = torch.arange(T, dtype=torch.int32, device="cuda")
    qo = torch.empty(T, Hq, D, device="cuda", dtype=torch.bfloat16)
    t = timed(lambda: hip.rope_kv(qkv, pos, slot, cs, kc, vc, Hq, qo))
    report("rope_kv", t, 2 * qkv.numel() * 2, None, T=T, Hq=Hq, Hkv=Hkv, D=D)


def bench_argmax(B, V=320):
    lg = torch.randn(B, V, device="cuda").to(torch.bfloat16)
    masks = torch.full((2, (V + 31) // 32), -1, dtype=torch.int32, device="cuda")
    mi = torch.zeros(B, dtype=torch.int32, device="cuda")
    out = torch.empty(B, dtype=torch.int32, device="cuda")
    t = timed(lambda: hip.masked_argmax(lg, masks, V, out, mi))
    report("masked_argmax", t, lg.numel() * 2, timed(lambda: lg.argmax(-1)), B=B, V=V)


def main() -> int:
    hip.lib()
    only = sys.argv[1] if len(sys.argv) > 1 else ""
    if only == "prefix8k":  # one case, for counter collection
        bench_prefix_attention(80, 8000, 100, max_seq=8192)
        return 0
    if only == "suffix":  # split size for the enrichment's short own-key suffixes
        for Ls in (300, 600, 900, 1500):
            for chunk in (256, 512, 1024):
                bench_prefix_attention(80, 4151, Ls, chunk=chunk)
        return 0
    if only in ("", "prefix"):
        bench_prefix_attention(80, 4151, 2500)
        bench_prefix_attention(256, 4151, 2500)
        bench_prefix_attention(16, 4151, 2500)
        bench_prefix_attention(80, 8000, 100, max_seq=8192)
        if only:
            return 0
    for B, L in ((1, 4096), (16, 2048), (64, 512), (64, 2300), (64, 4096), (256, 2300)):
        bench_decode_attention(B, L)
    bench_decode_attention(64, 2300, Hq=24, Hkv=8, D=128)
    for chunk in (128, 512, 1024):  # split size sweep
        for B, L in ((16, 2048), (64, 2300), (64, 4096)):
            bench_decode_attention(B, L, chunk=chunk, eager=False)
    for rows in (64, 256, 4096):
        bench_rmsnorm(rows)
        bench_silu(rows)
    for T in (64, 256, 2048):
        bench_rope(T)
    bench_argmax(256)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
