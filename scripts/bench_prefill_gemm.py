#!/usr/bin/env python3
"""Prefill-size GEMMs of dmcp-coder-1b (packed batched prefill, ~33k tokens)
through F.linear: hipBLASLt default heuristic vs PyTorch TunableOp (which
times every hipBLASLt / rocBLAS solution for the shape and keeps the
fastest).  Device time per call, TFLOP/s.

    python scripts/bench_prefill_gemm.py [M ...]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

SHAPES = {"qkv": (3072, 2048), "o": (2048, 2048), "gate_up": (16384, 2048), "down": (2048, 8192)}


def timed(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / iters * 1e-3


def main() -> int:
    rows = [int(x) for x in sys.argv[1:]] or [32768]
    tunable = os.environ.get("PYTORCH_TUNABLEOP_ENABLED") == "1"
    if tunable:
        torch.cuda.tunable.enable(True)
        torch.cuda.tunable.tuning_enable(True)
        torch.cuda.tunable.set_max_tuning_duration(200)
    for M in rows:
        for name, (N, K) in SHAPES.items():
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            w = torch.randn(N, K, device="cuda").to(torch.bfloat16)
            t0 = time.perf_counter()
            F.linear(x, w)  # the tuning call when enabled
            torch.cuda.synchronize()
            tune_s = time.perf_counter() - t0
            t = timed(lambda: F.linear(x, w))
            print(json.dumps({"gemm": name, "M": M, "N": N, "K": K, "tunable": tunable, "us": round(t * 1e6, 1),
                              "TFLOPs": round(2 * M * N * K / t / 1e12, 1), "first_call_s": round(tune_s, 2)}),
                  flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
