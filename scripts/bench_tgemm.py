"""Large-tile decode GEMM (csrc/tgemm.hip) against hipBLASLt (F.linear + the
unfused neighbour op) at the decode step's large row counts, per projection
of a preset's layer.  Weights rotate over copies larger than the 256 MB MALL
(a decode step streams 16 layers of distinct weights from HBM); each variant
is captured into one hipGraph of ``--reps`` launches and replayed, so the
numbers are device time.  Prints one JSON line per (rows, projection).

    python scripts/bench_tgemm.py --rows 520 640 768 1024 [--sweep]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from dmcp import ops  # noqa: E402
from dmcp.models.llm import preset  # noqa: E402
from dmcp.ops import hip  # noqa: E402


def graph_ms(fn, reps: int, copies: int) -> float:
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(2):
            fn(i % copies)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(reps):
            fn(i % copies)
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float("inf")
    for _ in range(5):
        t0.record()
        g.replay()
        t1.record()
        t1.synchronize()
        best = min(best, t0.elapsed_time(t1) / reps)
    return best


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="llama3.2-1b-code")
    ap.add_argument("--rows", type=int, nargs="+", default=[520, 640, 768, 1024])
    ap.add_argument("--reps", type=int, default=24)
    ap.add_argument("--sweep", action="store_true", help="also time every (S, mparts) around the plan")
    ap.add_argument("--only", default="", help="comma list of projections (qkv,o,gu,down,head)")
    ap.add_argument("--wg-sweep", action="store_true",
                    help="sweep the split count of the weight-streaming kernel's fused qkv / o / down ops")
    ap.add_argument("--fused-sweep", action="store_true",
                    help="sweep (S, mparts) of the FUSED op (GEMM + its reduction) for qkv / o / down")
    ap.add_argument("--copies", type=int, default=0, help="weight copies (default: enough to exceed 640 MB)")
    # 1 / 2: no refill DMA / no compute; 16-18: 64-B image rows; 32 / 34: a 2-stage ring;
    # 64-66: the register-weight kernel (full / no refill / no compute), 129 / 130: its weights 1 / 2 stages ahead;
    # 256: the plain kernel, 257-262: + weight L2 prefetch 1-6 stages ahead
    ap.add_argument("--probes", type=int, nargs="+", default=[1, 2, 16, 17, 18, 32, 34])
    ap.add_argument("--probe", action="store_true", help="also time the partials kernel without refill DMAs "
                    "(probe 1) and without compute (probe 2)")
    ap.add_argument("--probe-all", action="store_true", help="probes for gate/up and the head too (as plain "
                    "fp32-partials GEMMs of their shapes)")
    a = ap.parse_args()
    c = preset(a.preset)
    dev = "cuda"
    torch.manual_seed(0)
    H, I, Q = c.hidden, c.intermediate, c.qkv_dim
    shapes = {"qkv": (Q, H), "o": (H, H), "gu": (2 * I, H), "down": (H, I), "head": (c.vocab_size, H)}
    only = set(a.only.split(",")) if a.only else set(shapes)
    ws = torch.empty(16 * max(a.rows) * max(Q, H), dtype=torch.float32, device=dev)
    for M in a.rows:
        for name, (N, K) in shapes.items():
            if name not in only:
                continue
            copies = a.copies or max(1, min(8, -(-(640 << 20) // (N * K * 2))))
            Ws = [torch.randn(N, K, device=dev).mul_(0.02).to(torch.bfloat16) for _ in range(copies)]
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            flops = 2.0 * M * N * K
            rec = {"bench": "tgemm", "preset": a.preset, "rows": M, "proj": name, "N": N, "K": K,
                   "weight_copies": copies}
            if name == "head" and N % hip.TGEMM_NB:
                continue
            # correctness against F.linear (fp32 accumulate, bf16 out)
            ref = F.linear(x, Ws[0]).float()
            if name == "gu":
                got = hip.tgemm_swiglu(x, Ws[0]).float()
                exp = ops.silu_mul(F.linear(x, Ws[0])).float()
            elif name == "head":
                V = N
                masks = torch.full((1, (V + 31) // 32), -1, dtype=torch.int32, device=dev)
                midx = torch.zeros(M, dtype=torch.int32, device=dev)
                got = hip.tgemm_lm_head_argmax(x, Ws[0], masks, midx).long()
                exp = ref.argmax(-1)
                gv = ref.gather(1, got[:, None])[:, 0]
                rec["argmax_agree"] = float((got == exp).float().mean())
                rec["argmax_value_gap"] = float((ref.max(-1).values - gv).abs().max())
                got = exp = None
            else:
                S = hip.tgemm_partials(x, Ws[0], ws)
                got = ws[: S * M * N].view(S, M, N).sum(0)
                exp = ref
            if got is not None:
                rec["max_rel_err"] = float((got - exp).abs().max() / exp.abs().max().clamp_min(1e-6))
            # hipBLASLt (+ the unfused neighbour op of the step)
            if name == "gu":
                blas = lambda i: ops.silu_mul(F.linear(x, Ws[i]))  # noqa: E731
            elif name == "head":
                blas = lambda i: ops.masked_argmax(F.linear(x, Ws[i]), masks, vocab=N, mask_idx=midx)  # noqa: E731
            else:
                blas = lambda i: F.linear(x, Ws[i])  # noqa: E731
            rec["blas_us"] = round(graph_ms(blas, a.reps, copies) * 1e3, 2)
            mode = {"gu": "swiglu", "head": "argmax"}.get(name, "part")
            S0, mp0 = hip.tgemm_plan(M, N, K, mode)
            rec["plan"] = [S0, mp0]

            def run(S, mp):
                if name == "gu":
                    return lambda i: hip.tgemm_swiglu(x, Ws[i], mparts=mp)
                if name == "head":
                    return lambda i: hip.tgemm_lm_head_argmax(x, Ws[i], masks, midx, mparts=mp)
                return lambda i: hip.tgemm_partials(x, Ws[i], ws, splits=S, mparts=mp)
            rec["tgemm_us"] = round(graph_ms(run(S0, mp0), a.reps, copies) * 1e3, 2)
            if a.sweep:
                sw = {}
                mps = sorted({-(-M // 256), -(-M // 192), -(-M // 128), -(-M // 256) + 1, mp0})
                Ss = [1] if mode != "part" else sorted({1, 2, 3, 4, 6, 8, 10, 12, 16, S0})
                chunks = K // hip.TGEMM_KC
                for mp in mps:
                    if (-(-M // mp) + 15) // 16 * 16 > 256:
                        continue
                    for S in Ss:
                        if S > chunks or (S - 1) * -(-chunks // S) >= chunks:
                            continue
                        sw[f"S{S}_mp{mp}"] = round(graph_ms(run(S, mp), a.reps, copies) * 1e3, 2)
                rec["sweep_us"] = sw
                rec["sweep_best"] = min(sw.items(), key=lambda kv: kv[1])
            if a.probe and (mode == "part" or a.probe_all):
                # the probes write fp32 partials: the plan's (S, parts) for "part", (1, parts) otherwise
                pws = ws if mode == "part" else torch.empty(M * N, dtype=torch.float32, device=dev)
                Sp = S0 if mode == "part" else 1
                for pr in a.probes:
                    def probe(i, pr=pr):
                        hip._check(hip.lib().dmcp_tgemm_probe(pr, hip._ptr(x), hip._ptr(Ws[i]), hip._ptr(pws), M, N,
                                                              K, Sp, mp0, hip._stream()), "dmcp_tgemm_probe")
                    rec[f"probe{pr}_us"] = round(graph_ms(probe, a.reps, copies) * 1e3, 2)
                del pws
            # the fused op of the step vs hipBLASLt + the unfused neighbour op
            if name in ("o", "down"):
                resid = torch.randn(M, N, device=dev).to(torch.bfloat16)
                nw = torch.ones(N, device=dev, dtype=torch.bfloat16)
                rec["blas_fused_us"] = round(graph_ms(lambda i: ops.add_rmsnorm(F.linear(x, Ws[i]), nw, 1e-5,
                                                                                  residual=resid), a.reps, copies) * 1e3, 2)
                rec["fused_us"] = round(graph_ms(lambda i: hip.tgemm_resid_norm(x, Ws[i], resid, nw, 1e-5, ws),
                                                 a.reps, copies) * 1e3, 2)
                ho = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            elif name == "qkv":
                Hkv, D = c.n_kv_heads, c.head_dim
                kc = torch.zeros((8, Hkv, 2048, D), dtype=torch.uint8, device=dev)
                vc = torch.zeros_like(kc)
                pos = torch.arange(M, dtype=torch.int32, device=dev) % 2048
                sl = (torch.arange(M, dtype=torch.int32, device=dev) // 2048) % 8
                cs = ops.rope_tables(2048, D, c.rope_theta, device=dev).contiguous()
                rec["blas_fused_us"] = round(graph_ms(lambda i: ops.rope_kv(F.linear(x, Ws[i]), pos, sl, cs, kc, vc,
                                                                            c.n_heads), a.reps, copies) * 1e3, 2)
                rec["fused_us"] = round(graph_ms(lambda i: hip.tgemm_rope_kv(x, Ws[i], pos, sl, cs, kc, vc, c.n_heads,
                                                                             ws), a.reps, copies) * 1e3, 2)
                qo = torch.empty(M, c.n_heads, D, device=dev, dtype=torch.bfloat16)
            if M <= hip.WGEMM_MAX_ROWS and name != "head":  # the weight-streaming kernel's fused op
                wws = hip.wgemm_workspace(M, max(Q, H), dev)
                if name == "gu":
                    rec["wg_fused_us"] = round(graph_ms(lambda i: hip.wgemm_swiglu(x, Ws[i]), a.reps, copies) * 1e3, 2)
                elif name == "qkv":
                    rec["wg_fused_us"] = round(graph_ms(lambda i: hip.wgemm_rope_kv(x, Ws[i], pos, sl, cs, kc, vc,
                                                                                    c.n_heads, wws),
                                                        a.reps, copies) * 1e3, 2)
                else:
                    rec["wg_fused_us"] = round(graph_ms(lambda i: hip.wgemm_resid_norm(x, Ws[i], resid, nw, 1e-5, wws),
                                                        a.reps, copies) * 1e3, 2)
            elif M <= hip.WGEMM_MAX_ROWS and hip.lm_head_supported(N, K):
                rec["wg_fused_us"] = round(graph_ms(lambda i: hip.lm_head_argmax(x, Ws[i], masks, midx), a.reps,
                                                    copies) * 1e3, 2)
            if a.wg_sweep and M <= hip.WGEMM_MAX_ROWS and name in ("qkv", "o", "down"):
                # the weight-streaming kernel's fused op over its split count (the plan's S is wg_plan)
                rec["wg_plan"] = list(hip.wgemm_plan(M, N, K))
                sws = hip.wgemm_workspace(4 * M, max(Q, H), dev)  # room for 32 slices
                wsw = {}
                for S in (1, 2, 4, 8, 16, 32):
                    if K % (64 * S):
                        continue
                    if name == "qkv":
                        f = lambda i, S=S: hip.wgemm_rope_kv(x, Ws[i], pos, sl, cs, kc, vc, c.n_heads, sws,  # noqa
                                                             splits=S)
                    else:
                        f = lambda i, S=S: hip.wgemm_resid_norm(x, Ws[i], resid, nw, 1e-5, sws, splits=S)  # noqa
                    wsw[f"S{S}"] = round(graph_ms(f, a.reps, copies) * 1e3, 2)
                rec["wg_sweep_us"] = wsw
                rec["wg_sweep_best"] = min(wsw.items(), key=lambda kv: kv[1])
            if a.fused_sweep and name in ("qkv", "o", "down"):
                fsw = {}
                chunks = K // hip.TGEMM_KC
                for mp in sorted({-(-M // 256), -(-M // 192), -(-M // 128), -(-M // 96), -(-M // 64)}):
                    if (-(-M // mp) + 15) // 16 * 16 > 256:
                        continue
                    for S in (1, 2, 3, 4, 5, 6, 8, 10, 12):
                        if S > chunks or (S - 1) * -(-chunks // S) >= chunks:
                            continue
                        if name == "qkv":
                            f = lambda i, S=S, mp=mp: (hip.tgemm_partials(x, Ws[i], ws, splits=S, mparts=mp),  # noqa
                                                       hip._check(hip.lib().dmcp_reduce_rope_kv(
                                                           hip._ptr(ws), S, hip._ptr(pos), hip._ptr(sl), hip._ptr(cs),
                                                           hip._ptr(qo), hip._ptr(kc), hip._ptr(vc), M, c.n_heads, Hkv,
                                                           D, 2048, cs.shape[0], 8, 1, hip._stream()), "reduce"))
                        else:
                            f = lambda i, S=S, mp=mp: (hip.tgemm_partials(x, Ws[i], ws, splits=S, mparts=mp),  # noqa
                                                       hip._check(hip.lib().dmcp_reduce_resid_norm(
                                                           hip._ptr(ws), S, hip._ptr(resid), hip._ptr(nw), hip._ptr(ho),
                                                           M, N, 1e-5, hip._stream()), "reduce"))
                        fsw[f"S{S}_mp{mp}"] = round(graph_ms(f, a.reps, copies) * 1e3, 2)
                rec["fused_sweep_us"] = fsw
                rec["fused_sweep_best"] = min(fsw.items(), key=lambda kv: kv[1])
            rec["tgemm_pflops"] = round(flops / (rec["tgemm_us"] * 1e-6) / 1e15, 3)
            rec["blas_pflops"] = round(flops / (rec["blas_us"] * 1e-6) / 1e15, 3)
            print(json.dumps(rec), flush=True)
            del Ws
            torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
