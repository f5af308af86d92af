#!/usr/bin/env python3
"""Weight-streaming GEMM (csrc/wgemm.hip) alone at decode-step shapes of
dmcp-coder-1b: device time per call with 8 weight copies cycled inside one
hipGraph (so weights stream from HBM as in the step, not from MALL), and the
effective weight bandwidth.

    python scripts/bench_wgemm.py [M ...] > gpurun_out/wgemm.jsonl
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dmcp.ops import hip  # noqa: E402
from scripts.bench_kernels import timed  # noqa: E402

COPIES = 8
SHAPES = {"qkv": (3072, 2048, "part"), "o": (2048, 2048, "part"), "gate_up": (16384, 2048, "swiglu"),
          "down": (2048, 8192, "part")}


def main() -> int:
    rows = [int(a) for a in sys.argv[1:]] or [78, 320, 512]
    for M in rows:
        for name, (N, K, kind) in SHAPES.items():
            ws = [torch.randn(N, K, device="cuda").to(torch.bfloat16) for _ in range(COPIES)]
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            ws_part = hip.wgemm_workspace(M, max(N, 8192), x.device)
            out = torch.empty(M, N // 2, device="cuda", dtype=torch.bfloat16)
            if kind == "swiglu":
                def fn():
                    for w in ws:
                        hip.wgemm_swiglu(x, w, out)
            else:
                def fn():
                    for w in ws:
                        hip.wgemm_partials(x, w, ws_part)
            t = timed(fn, iters=10) / COPIES
            S, mparts = hip.wgemm_plan(M, N, K, swiglu=kind == "swiglu")
            print(json.dumps({"gemm": name, "M": M, "N": N, "K": K, "S": S, "mparts": mparts, "us": round(t * 1e6, 2),
                              "weight_TBps": round(N * K * 2 / t / 1e12, 2),
                              "TFLOPs": round(2 * M * N * K / t / 1e12, 1),
                              "dbg": os.environ.get("DMCP_WG_DBG", "0")}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
