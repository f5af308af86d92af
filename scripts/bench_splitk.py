#!/usr/bin/env python3
"""O / down projection + residual add + RMSNorm at decode row counts:
F.linear (hipBLASLt) + add_rmsnorm vs linear_resid_norm (csrc/splitk_gemm.hip),
16 distinct weight copies cycled (weights stream from HBM).  One JSON line
per (op, M, arm[, splits])."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from dmcp.ops import hip  # noqa: E402
from scripts.bench_kernels import timed  # noqa: E402

SHAPES = {"o": (2048, 2048), "down": (2048, 8192)}
LAYERS = 16


def main() -> int:
    torch.manual_seed(0)
    for name, (N, K) in SHAPES.items():
        ws_w = [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(LAYERS)]
        g = torch.ones(N, dtype=torch.bfloat16, device="cuda")
        for M in (48, 78, 96, 128):
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            resid = torch.randn(M, N, device="cuda").to(torch.bfloat16)
            ws = torch.empty(32 * M * N, dtype=torch.float32, device="cuda")

            def ref():
                for w in ws_w:
                    o = F.linear(x, w)
                    hip.add_rmsnorm(o, g, 1e-5, residual=resid)
            t = timed(ref, iters=4) / LAYERS
            print(json.dumps({"op": name, "M": M, "arm": "hipblaslt+add_rmsnorm", "us": round(t * 1e6, 2),
                              "weight_TBps": round(N * K * 2 / t / 1e12, 2)}), flush=True)
            for variant in (0, 1):
                for S in (0, 4, 8, 16):
                    Sx = S or hip.splitk_splits(N, K)
                    if K % ((128 if variant else 32) * Sx):
                        continue

                    def mine(S=S, variant=variant):
                        for w in ws_w:
                            hip.linear_resid_norm(x, w, resid, g, 1e-5, ws, splits=S, variant=variant)
                    t = timed(mine, iters=4) / LAYERS
                    print(json.dumps({"op": name, "M": M, "arm": f"splitk_v{variant}", "splits": Sx, "auto": S == 0,
                                      "us": round(t * 1e6, 2), "weight_TBps": round(N * K * 2 / t / 1e12, 2)}),
                          flush=True)
    # QKV projection + RoPE + KV append (dmcp-coder-1b heads, fp8 cache)
    from dmcp.ops import reference
    Hq, Hkv, D, K = 32, 8, 64, 2048
    N = (Hq + 2 * Hkv) * D
    ws_w = [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(LAYERS)]
    cs = reference.rope_tables(4096, D, device="cuda")
    kc = torch.zeros(256, Hkv, 4096, D, dtype=torch.uint8, device="cuda")
    vc = torch.zeros_like(kc)
    for M in (48, 78, 96, 128):
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        pos = torch.arange(M, dtype=torch.int32, device="cuda") + 1000
        slot = torch.arange(M, dtype=torch.int32, device="cuda")
        ws = torch.empty(32 * M * N, dtype=torch.float32, device="cuda")

        def ref():
            for w in ws_w:
                hip.rope_kv(F.linear(x, w), pos, slot, cs, kc, vc, Hq)
        t = timed(ref, iters=4) / LAYERS
        print(json.dumps({"op": "qkv_rope", "M": M, "arm": "hipblaslt+rope_kv", "us": round(t * 1e6, 2),
                          "weight_TBps": round(N * K * 2 / t / 1e12, 2)}), flush=True)
        for S in (0, 4):
            Sx = S or hip.splitk_splits(N, K)

            def mine(S=S):
                for w in ws_w:
                    hip.linear_rope_kv(x, w, pos, slot, cs, kc, vc, Hq, ws, splits=S)
            t = timed(mine, iters=4) / LAYERS
            print(json.dumps({"op": "qkv_rope", "M": M, "arm": "splitk_v1", "splits": Sx, "us": round(t * 1e6, 2),
                              "weight_TBps": round(N * K * 2 / t / 1e12, 2)}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
