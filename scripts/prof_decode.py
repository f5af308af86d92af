#!/usr/bin/env python3
"""Standalone decode-attention driver for rocprofv3 (kernel trace / PMC runs).

    rocprofv3 --kernel-trace --stats -d gpurun_out/pd -o pd -- python3 scripts/prof_decode.py --B 64 --L 512
"""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dmcp.ops import hip  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--L", type=int, default=512)
    ap.add_argument("--Hq", type=int, default=32)
    ap.add_argument("--Hkv", type=int, default=8)
    ap.add_argument("--D", type=int, default=64)
    ap.add_argument("--max-seq", type=int, default=4096)
    ap.add_argument("--chunk", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    hip.lib()
    dev = "cuda"
    kc = torch.randn(a.B, a.Hkv, a.max_seq, a.D, device=dev).to(torch.bfloat16)
    vc = torch.randn_like(kc)
    q = torch.randn(a.B, a.Hq, a.D, device=dev).to(torch.bfloat16)
    slot = torch.arange(a.B, dtype=torch.int32, device=dev)
    sl = torch.full((a.B,), a.L, dtype=torch.int32, device=dev)
    ws = hip.decode_workspace(a.B, a.Hq, a.Hkv, a.D, a.max_seq, dev, a.chunk)
    out = torch.empty_like(q)
    for _ in range(a.iters):
        hip.decode_attention(q, kc, vc, slot, sl, 1 / math.sqrt(a.D), workspace=ws, chunk=a.chunk, out=out)
    torch.cuda.synchronize()
    print("ok", float(out.float().abs().sum()))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
