#!/usr/bin/env python3
"""Fused decode GEMMs (csrc/fused_gemm.hip) vs hipBLASLt at decode shapes of
dmcp-coder-1b: device time per call (hipGraph-replayed, weights of 16 layers
cycled so they stream from HBM as in a real step) and achieved weight
bandwidth.  One JSON line per (op, M, wk).

    python scripts/bench_fused.py > gpurun_out/fused.jsonl
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from dmcp.ops import hip, reference  # noqa: E402
from scripts.bench_kernels import timed  # noqa: E402

H, I, HQ, HKV, D, LAYERS = 2048, 8192, 32, 8, 64, 16


def main() -> int:
    hip.lib()
    dev = "cuda"
    shapes = {"qkv": ((HQ + 2 * HKV) * D, H), "o": (H, HQ * D), "gate_up": (2 * I, H), "down": (H, I),
              "lm_head": (320, H)}
    ws = {k: [torch.randn(n, kk, device=dev).mul_(0.02).to(torch.bfloat16) for _ in range(LAYERS)]
          for k, (n, kk) in shapes.items()}
    cs = reference.rope_tables(8192, D, device=dev)
    kc = torch.zeros(65, HKV, 1024, D, dtype=torch.bfloat16, device=dev)
    vc = torch.zeros_like(kc)
    for M in (16, 32, 64, 96, 128):
        x2 = torch.randn(M, H, device=dev).to(torch.bfloat16)
        x8 = torch.randn(M, I, device=dev).to(torch.bfloat16)
        r = torch.randn(M, H, device=dev).to(torch.bfloat16)
        pos = torch.arange(M, dtype=torch.int32, device=dev)
        slot = (torch.arange(M, dtype=torch.int32, device=dev) % 64)
        ctr = [0]

        def nxt(name):
            ctr[0] += 1
            return ws[name][ctr[0] % LAYERS]
        for wk in (4, 8, 16):
            cases = {
                "qkv": lambda: hip.fused_rope_kv(x2, nxt("qkv"), 1e-5, pos, slot, cs, kc, vc, HQ, wk=wk),
                "o": lambda: hip.fused_resid(x2, nxt("o"), r, wk=wk),
                "gate_up": lambda: hip.fused_swiglu(x2, nxt("gate_up"), 1e-5, wk=wk),
                "down": lambda: hip.fused_resid(x8, nxt("down"), r, wk=wk),
                "lm_head": lambda: hip.fused_linear_norm(x2, nxt("lm_head"), 1e-5, wk=wk),
            }
            for name, fn in cases.items():
                t = timed(fn, iters=32)
                n, k = shapes[name]
                print(json.dumps({"op": name, "impl": "fused", "M": M, "wk": wk, "us": round(t * 1e6, 2),
                                  "weight_TBps": round(n * k * 2 / t / 1e12, 2)}), flush=True)
        for name, (n, k) in shapes.items():
            x = x8 if name == "down" else x2
            t = timed(lambda: F.linear(x, nxt(name)), iters=32)
            print(json.dumps({"op": name, "impl": "hipblaslt", "M": M, "us": round(t * 1e6, 2),
                              "weight_TBps": round(n * k * 2 / t / 1e12, 2)}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
