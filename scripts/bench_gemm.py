#!/usr/bin/env python3
"""Decode-step GEMM shapes of dmcp-coder-1b through F.linear (hipBLASLt):
time per call (hipGraph-replayed) and achieved weight bandwidth.  M = rows of
a decode step (~80 with jump-forward), weights [N, K] bf16 read once per call.

    python scripts/bench_gemm.py > gpurun_out/gemm.jsonl
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from scripts.bench_kernels import timed  # noqa: E402

SHAPES = {"qkv": (3072, 2048), "o": (2048, 2048), "gate_up": (16384, 2048), "down": (2048, 8192),
          "lm_head": (320, 2048)}


def main() -> int:
    for M in (16, 64, 80, 128, 256):
        for name, (N, K) in SHAPES.items():
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            w = torch.randn(N, K, device="cuda").to(torch.bfloat16)
            out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            t = timed(lambda: torch.matmul(x, w.t(), out=out))
            nbytes = (N * K + M * K + M * N) * 2
            print(json.dumps({"gemm": name, "M": M, "N": N, "K": K, "us": round(t * 1e6, 2),
                              "GBps": round(nbytes / t / 1e9, 1), "pct_hbm_peak": round(100 * nbytes / t / 8e12, 1),
                              "TFLOPs": round(2 * M * N * K / t / 1e12, 1)}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
