"""The fused split-K GEMMs of the > 512-row decode step (csrc/tgemm.hip TgEpi:
last-arriver fixup, RMSNorm row scale) against the round-5 pair they
replace (split-K partials + wgemm.hip's reduction kernel), per projection of
a preset's layer, with a (S, M parts) sweep of the new ones.  Weights rotate
over copies larger than the MALL; device time of hipGraph replays.  One JSON
line per (rows, projection).

    python scripts/bench_tgemm_fixup.py --rows 520 610 768 1024 [--sweep]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dmcp import ops  # noqa: E402
from dmcp.models.llm import preset  # noqa: E402
from dmcp.ops import hip  # noqa: E402
from scripts.bench_tgemm import graph_ms  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="llama3.2-1b-code")
    ap.add_argument("--rows", type=int, nargs="+", default=[520, 610, 768, 1024])
    ap.add_argument("--reps", type=int, default=24)
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--only", default="qkv,o,down,gu")
    a = ap.parse_args()
    c = preset(a.preset)
    dev = "cuda"
    torch.manual_seed(0)
    H, I, Q, D, Hkv = c.hidden, c.intermediate, c.qkv_dim, c.head_dim, c.n_kv_heads
    shapes = {"qkv": (Q, H), "o": (H, H), "down": (H, I), "gu": (2 * I, H)}
    only = set(a.only.split(","))
    old_ws = torch.empty(16 * max(a.rows) * max(Q, H), dtype=torch.float32, device=dev)
    fx = hip.tgemm_fixup_workspace(max(a.rows), max(Q, H), H, dev)
    kc = torch.zeros((8, Hkv, 2048, D), dtype=torch.uint8, device=dev)
    vc = torch.zeros_like(kc)
    cs = ops.rope_tables(2048, D, c.rope_theta, device=dev).contiguous()
    nw = torch.ones(H, device=dev, dtype=torch.bfloat16)
    for M in a.rows:
        pos = torch.arange(M, dtype=torch.int32, device=dev) % 2048
        sl = (torch.arange(M, dtype=torch.int32, device=dev) // 2048) % 8
        sq = torch.rand((H // 256, M), device=dev) * 100
        rs = hip.RowScale(sq, H, 1e-5)
        resid = torch.randn(M, H, device=dev).to(torch.bfloat16)
        for name, (N, K) in shapes.items():
            if name not in only:
                continue
            copies = max(1, min(8, -(-(640 << 20) // (N * K * 2))))
            Ws = [torch.randn(N, K, device=dev).mul_(0.02).to(torch.bfloat16) for _ in range(copies)]
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            rec = {"bench": "tgemm_fixup", "preset": a.preset, "rows": M, "proj": name, "N": N, "K": K}
            if name == "qkv":
                old = lambda i: hip.tgemm_rope_kv(x, Ws[i], pos, sl, cs, kc, vc, c.n_heads, old_ws)  # noqa: E731

                def new(i, S=0, mp=0):
                    return hip.tgemm_qkv(x, Ws[i], pos, sl, cs, kc, vc, c.n_heads, fx, row_scale=rs, splits=S,
                                         mparts=mp)
            elif name == "gu":
                old = lambda i: hip.tgemm_swiglu(x, Ws[i])  # noqa: E731

                def new(i, S=0, mp=0):
                    return hip.tgemm_swiglu_scaled(x, Ws[i], rs, mparts=mp)
            else:
                old = lambda i: hip.tgemm_resid_norm(x, Ws[i], resid, nw, 1e-5, old_ws)  # noqa: E731

                def new(i, S=0, mp=0):
                    return hip.tgemm_resid(x, Ws[i], resid, fx, 1e-5, splits=S, mparts=mp)
            rec["old_us"] = round(graph_ms(old, a.reps, copies) * 1e3, 2)
            rec["plan"] = list(hip.tgemm_fixup_plan(M, N, K)) if name != "gu" else [1, hip.tgemm_plan(M, N, K,
                                                                                                     "swiglu")[1]]
            rec["new_us"] = round(graph_ms(new, a.reps, copies) * 1e3, 2)
            if a.sweep and name != "gu":
                sw = {}
                chunks = K // hip.TGEMM_KC
                for mp in sorted({-(-M // r) for r in (256, 192, 128, 96, 64)}):
                    if (-(-M // mp) + 15) // 16 * 16 > 256:
                        continue
                    for S in (1, 2, 3, 4, 5, 6, 8, 10, 12):
                        if S > chunks or (S - 1) * -(-chunks // S) >= chunks:
                            continue
                        sw[f"S{S}_mp{mp}"] = round(graph_ms(lambda i, S=S, mp=mp: new(i, S, mp), a.reps, copies)
                                                   * 1e3, 2)
                rec["sweep_us"] = sw
                rec["sweep_best"] = min(sw.items(), key=lambda kv: kv[1])
            print(json.dumps(rec), flush=True)
            del Ws
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
