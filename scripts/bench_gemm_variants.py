#!/usr/bin/env python3
"""Decode-step weight GEMMs of dmcp-coder-1b, library formulations A/B (GPU box).

Every op cycles through 16 distinct weight copies (one per layer), as a
decode step does, so the weights stream from HBM instead of sitting in the
256 MB MALL.  Arms: hipBLASLt x @ W^T (the model's F.linear), the same
product on PyTorch's other ROCm BLAS back-ends ("hipblas" = rocBLAS, "ck" =
composable_kernel), and the transposed problem W @ x^T (hipBLASLt picks other
kernels for a wide-N, skinny-M output).  One JSON line per (op, M, arm).

    python scripts/bench_gemm_variants.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from scripts.bench_kernels import timed  # noqa: E402

SHAPES = {"qkv": (3072, 2048), "o": (2048, 2048), "gate_up": (16384, 2048), "down": (2048, 8192)}
LAYERS = 16


def main() -> int:
    torch.manual_seed(0)
    ws = {name: [torch.randn(N, K, device="cuda").to(torch.bfloat16) for _ in range(LAYERS)]
          for name, (N, K) in SHAPES.items()}
    for M in (78, 96, 128):
        for name, (N, K) in SHAPES.items():
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            out_t = torch.empty(N, M, device="cuda", dtype=torch.bfloat16)
            xt = x.t().contiguous()
            arms = {}

            def lt():
                for w in ws[name]:
                    torch.matmul(x, w.t(), out=out)
            arms["hipblaslt"] = lt

            def tr():
                for w in ws[name]:
                    torch.matmul(w, xt, out=out_t)
            arms["hipblaslt_transposed"] = tr
            res = {}
            for arm, fn in arms.items():
                res[arm] = timed(fn, iters=4) / LAYERS
            prev = torch.backends.cuda.preferred_blas_library()
            for lib in ("hipblas", "ck"):  # "hipblas" = the rocBLAS path on ROCm builds
                try:
                    torch.backends.cuda.preferred_blas_library(lib)
                    res[lib] = timed(lt, iters=4) / LAYERS
                except Exception as e:  # backend unavailable on this build
                    print(json.dumps({"lib": lib, "error": str(e)[:200]}), flush=True)
                finally:
                    torch.backends.cuda.preferred_blas_library(prev)
            for arm, t in res.items():
                print(json.dumps({"gemm": name, "M": M, "N": N, "K": K, "arm": arm, "us": round(t * 1e6, 2),
                                  "weight_TBps": round(N * K * 2 / t / 1e12, 2)}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
