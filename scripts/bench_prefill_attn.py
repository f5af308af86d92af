#!/usr/bin/env python3
"""Prefill attention alone (GPU box): the MFMA kernel (csrc/prefill_attn.hip,
variants, split-K 1/2/4) against the SDPA + log-sum-exp path it replaced, on the
enrichment shape -- one class's own tokens (--tokens) after a shared prefix
(--prefix) read from another slot.  Interleaved A/B, one JSON line per arm:
us per call and attention TFLOP/s (4 * Hq * D * T * (P + T/2) FLOPs).

    python scripts/bench_prefill_attn.py [--heads 32 --kv-heads 8 --dim 64]
"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--prefix", type=int, default=4151)
    ap.add_argument("--tokens", type=int, default=2100)
    ap.add_argument("--heads", type=int, default=32)
    ap.add_argument("--kv-heads", type=int, default=8)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--arms", default="", help="comma-separated arm names to run (default: all)")
    a = ap.parse_args()
    from dmcp.models.llm import _extend_attention
    from dmcp.ops import hip
    hip.lib()
    D, Hq, Hkv, P, T = a.dim, a.heads, a.kv_heads, a.prefix, a.tokens
    MAXS = P + T + 64
    g = torch.Generator(device="cuda").manual_seed(0)
    kc = torch.randn(2, Hkv, MAXS, D, generator=g, device="cuda").to(torch.bfloat16)
    vc = torch.randn(2, Hkv, MAXS, D, generator=g, device="cuda").to(torch.bfloat16)
    q = torch.randn(T, Hq, D, generator=g, device="cuda").to(torch.bfloat16)
    kc[0, :, :P] = kc[1, :, :P]  # slot 0 also holds the prefix (what the SDPA path reads)
    vc[0, :, :P] = vc[1, :, :P]
    scale = 1 / math.sqrt(D)
    flops = 4 * Hq * D * T * (P + T / 2)

    def sdpa():
        k = kc[0, :, :P + T].unsqueeze(0)
        v = vc[0, :, :P + T].unsqueeze(0)
        return _extend_attention(q.transpose(0, 1).unsqueeze(0), k, v, P, scale)[0].transpose(0, 1)

    arms = {"sdpa": sdpa}
    for variant in hip.PREFILL_VARIANTS[D]:
        for nsplit in (1, 2, 4):
            arms[f"mfma_v{variant}_s{nsplit}"] = (lambda v, n: lambda: hip.prefill_attention(
                q, kc, vc, 0, P, 1, P, scale, variant=v, nsplit=n))(variant, nsplit)
    if a.arms:
        keep = set(a.arms.split(","))
        arms = {k: v for k, v in arms.items() if k in keep}
    ref = sdpa().float()
    for name, fn in arms.items():
        err = (fn().float() - ref).abs().max().item()
        print(json.dumps({"arm": name, "max_abs_err_vs_sdpa": round(err, 5)}), flush=True)
    times = {k: [] for k in arms}
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(a.rounds):
        for name, fn in arms.items():
            fn()
            ev0.record()
            for _ in range(a.iters):
                fn()
            ev1.record()
            ev1.synchronize()
            times[name].append(ev0.elapsed_time(ev1) / a.iters * 1e3)
    for name, ts in times.items():
        us = sorted(ts)[len(ts) // 2]
        print(json.dumps({"bench": "prefill_attn", "arm": name, "T": T, "P": P, "Hq": Hq, "Hkv": Hkv, "D": D,
                          "us": round(us, 1), "TFLOPs": round(flops / us / 1e6, 1)}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
