"""Shared-prefix decode attention (prefill_attn.hip in prefix mode) in
isolation: every row attends the P-key shared prefix plus ``--own`` keys of
its own slot.  Times the decode_attention call with the prefix at length P
and at length 0 (the same graph: the length lives in device memory, so the
prefix blocks exit at once) and reports the difference as the prefix
kernel's time and its TFLOP/s (4 B Hq P D flops: QK^T + PV).  One JSON line
per (rows, P); run under rocprofv3 --kernel-trace --stats for the per-kernel
split.

    python scripts/bench_prefix.py --rows 320 512 610 --prefix 1119 4949
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dmcp.ops import hip  # noqa: E402
from dmcp.ops.reference import SharedPrefix  # noqa: E402


def timed_us(fn, iters=20) -> float:
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
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
    best = float("inf")
    for _ in range(5):
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) * 1e3 / iters)
    return best


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, nargs="+", default=[320, 512, 610])
    ap.add_argument("--prefix", type=int, nargs="+", default=[1119, 4949])
    ap.add_argument("--own", type=int, default=64)
    ap.add_argument("--kv", choices=["bf16", "fp8"], default="fp8")
    ap.add_argument("--splits", type=int, nargs="*", default=[], help="DMCP_PREFIX_SPLITS values to sweep")
    a = ap.parse_args()
    Hq, Hkv, D, MAXS = 32, 8, 64, 8192
    dev = "cuda"
    torch.manual_seed(0)
    for B in a.rows:
        S = B + 1
        kc = (torch.randn(S, Hkv, MAXS, D, device=dev) * 0.5).to(torch.float8_e4m3fn)
        vc = (torch.randn(S, Hkv, MAXS, D, device=dev) * 0.5).to(torch.float8_e4m3fn)
        if a.kv == "fp8":
            kc, vc = kc.view(torch.uint8), vc.view(torch.uint8)
        else:
            kc, vc = kc.to(torch.bfloat16), vc.to(torch.bfloat16)
        q = torch.randn(B, Hq, D, device=dev).to(torch.bfloat16)
        slot = torch.arange(B, dtype=torch.int32, device=dev)
        out = torch.empty_like(q)
        for P in a.prefix:
            sl = torch.full((B,), P + a.own, dtype=torch.int32, device=dev)
            plen = torch.tensor([P], dtype=torch.int32, device=dev)
            pre = SharedPrefix(kc[B], vc[B], plen)
            ws = hip.decode_workspace(B, Hq, Hkv, D, MAXS, dev, 256, hip.PREFIX_MFMA_MAX_SPLITS)
            rec = {"bench": "prefix_attention", "rows": B, "P": P, "own": a.own, "kv": a.kv}
            for sp in [None] + list(a.splits):
                if sp is not None:
                    os.environ["DMCP_PREFIX_SPLITS"] = str(sp)
                else:
                    os.environ.pop("DMCP_PREFIX_SPLITS", None)
                fn = lambda: hip.decode_attention(q, kc, vc, slot, sl, 1 / math.sqrt(D), workspace=ws,  # noqa: E731
                                                  out=out, prefix=pre)
                plen.fill_(P)
                sl.fill_(P + a.own)
                t1 = timed_us(fn)
                plen.fill_(0)  # same launches, the prefix blocks exit at once; rows keep only their own keys
                sl.fill_(a.own)
                t0 = timed_us(fn)
                plen.fill_(P)
                sl.fill_(P + a.own)
                tp = max(1e-3, t1 - t0)
                key = "" if sp is None else f"_sp{sp}"
                rec["splits" + key] = hip.prefix_mfma_splits(B, Hq // Hkv, Hkv)
                rec["total_us" + key] = round(t1, 2)
                rec["no_prefix_us" + key] = round(t0, 2)
                rec["prefix_us" + key] = round(tp, 2)
                rec["prefix_tflops" + key] = round(4.0 * B * Hq * P * D / (tp * 1e-6) / 1e12, 1)
            os.environ.pop("DMCP_PREFIX_SPLITS", None)
            print(json.dumps(rec), flush=True)
        del kc, vc
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
