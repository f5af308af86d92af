"""The batched prefill's attention at the engine's shapes (GPU box):
``hip.prefill_attention_varlen`` over N packed sequences of T own tokens
after a P-token shared prefix read in place from its own slot, fp8 (e4m3)
or bf16 KV caches, against the same sequences one ``prefill_attention``
launch each.  Graph-free event timing (one call is ~100 us - ms).  Prints
us per call and attention TFLOP/s (4 * Hq * D * T * (P + T/2) per sequence).

  python scripts/bench_varlen_attn.py [--seqs 45 --tokens 1003 --prefix 4949 --kv fp8]
"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seqs", type=int, default=45)
    ap.add_argument("--tokens", type=int, default=1003)
    ap.add_argument("--prefix", type=int, default=4949)
    ap.add_argument("--heads", type=int, default=32)
    ap.add_argument("--kv-heads", type=int, default=8)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--kv", default="fp8", choices=["fp8", "bf16"])
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    import torch
    from dmcp.ops import hip
    N, T, P, Hq, Hkv, D = args.seqs, args.tokens, args.prefix, args.heads, args.kv_heads, args.dim
    S = N + 1
    MAXS = P + T + 64
    g = torch.Generator(device="cuda").manual_seed(0)
    if args.kv == "fp8":
        kc = torch.randint(0, 256, (S, Hkv, MAXS, D), device="cuda", dtype=torch.uint8, generator=g)
        vc = torch.randint(0, 256, (S, Hkv, MAXS, D), device="cuda", dtype=torch.uint8, generator=g)
        kc &= 0x77  # finite e4m3 values of moderate size (no NaN pattern, |x| <= 1.75 * 2^6)
        vc &= 0x77
    else:
        kc = torch.randn(S, Hkv, MAXS, D, device="cuda", generator=g).to(torch.bfloat16)
        vc = torch.randn(S, Hkv, MAXS, D, device="cuda", generator=g).to(torch.bfloat16)
    q = torch.randn(N * T, Hq, D, device="cuda", generator=g).to(torch.bfloat16)
    prefix_slot = N
    offsets = [i * T for i in range(N + 1)]
    slots = list(range(N))
    starts = [P] * N
    shared = [P] * N
    scale = 1 / math.sqrt(D)
    flops = N * 4 * Hq * D * T * (P + T / 2)

    def varlen():
        return hip.prefill_attention_varlen(q, kc, vc, offsets, slots, starts, prefix_slot, shared, scale)

    def per_seq():
        for i in range(N):
            hip.prefill_attention(q[i * T:(i + 1) * T], kc, vc, i, P, prefix_slot, P, scale)

    out = {}
    for name, fn in (("varlen", varlen), ("per_seq", per_seq)):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / args.iters
        out[name] = us
        print(json.dumps({"bench": "varlen_attn", "arm": name, "seqs": N, "T": T, "P": P, "kv": args.kv, "D": D,
                          "us": round(us, 1), "TFLOPs": round(flops / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
