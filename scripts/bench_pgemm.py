#!/usr/bin/env python3
"""The four prefill projections of a model preset at a prefill batch's row
count (GPU box): the MXFP8 kernels of csrc/pgemm.hip (with their fused
epilogues) against hipBLASLt's bf16 F.linear (+ the unfused epilogue ops the
bf16 prefill runs) -- and torch._scaled_mm fp8 when this torch build has it.
Prints one JSON line per (projection, implementation): us and TFLOP/s.

    python scripts/bench_pgemm.py --preset llama3.2-1b-code --rows 24576
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def timed_graph(fn, iters):
    """Device time of fn captured in a hipGraph (the decode step runs that
    way): eager calls of the small decode GEMMs are host-launch-bound."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(10):
            fn()
    return timed(g.replay, max(1, iters // 10)) / 10


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="llama3.2-1b-code")
    ap.add_argument("--rows", type=int, default=24576)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--decode-rows", type=int, nargs="*", default=[78, 320, 512])
    ap.add_argument("--waves", type=int, default=0, choices=[0, 4, 8],
                    help="waves per block of the MX prefill GEMM (0: the library default)")
    ap.add_argument("--bk", type=int, default=0, choices=[0, 64, 128],
                    help="K per LDS stage of the MX prefill GEMM (0: the library default)")
    ap.add_argument("--group", type=int, default=0, help="M tiles per block-order group (0: the library default)")
    ap.add_argument("--areg", type=int, default=-1, choices=[-1, 0, 1],
                    help="A operand through registers in the 128-deep kernel (-1: the library default)")
    a = ap.parse_args()
    from dmcp import ops
    from dmcp.models.llm import preset
    from dmcp.ops import hip, reference as R
    if a.waves:
        hip.pgemm_set_waves(a.waves)
    if a.bk:
        hip.pgemm_set_bk(a.bk)
    if a.group:
        hip.pgemm_set_group(a.group)
    if a.areg >= 0:
        hip.pgemm_set_areg(a.areg)
    c = preset(a.preset)
    M, H, I, D = a.rows, c.hidden, c.intermediate, c.head_dim
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)

    def bf(*s, scale=1.0):
        return (torch.randn(*s, generator=g, device=dev) * scale).to(torch.bfloat16)
    shapes = {"qkv": (c.qkv_dim, H), "o": (H, c.n_heads * D), "gate_up": (2 * I, H), "down": (H, I)}
    x = {k: bf(M, K, scale=2.0) for k, (N, K) in shapes.items()}
    w = {k: bf(N, K, scale=0.03) for k, (N, K) in shapes.items()}
    w8 = {k: R.quantize_weight(v) for k, v in w.items()}
    mx = {k: ops.mx_quant(v) for k, v in x.items()}
    S, MAXS = 64, 2048
    kc = torch.zeros(S, c.n_kv_heads, MAXS, D, dtype=torch.uint8, device=dev)
    vc = torch.zeros_like(kc)
    cos_sin = R.rope_tables(MAXS, D, c.rope_theta, dev)
    pos = (torch.arange(M, device=dev, dtype=torch.int32) % MAXS)
    slot = (torch.arange(M, device=dev, dtype=torch.int32) // MAXS) % S
    resid = bf(M, H)
    out = {}

    def line(name, impl, us, N, K):
        tf = 2.0 * M * N * K / us / 1e6
        out.setdefault(name, {})[impl] = us
        print(json.dumps({"proj": name, "impl": impl, "rows": M, "N": N, "K": K, "us": round(us, 1),
                          "tflops": round(tf, 1)}), flush=True)

    for name, (N, K) in shapes.items():
        aq, as_ = mx[name]
        wq, ws = w8[name]
        line(name, "bf16_hipblaslt", timed(lambda: F.linear(x[name], w[name]), a.iters), N, K)
        if name == "qkv":
            fn = lambda: ops.pgemm_qkv(aq, as_, wq, ws, pos, slot, cos_sin, kc, vc, c.n_heads)  # noqa: E731
        elif name == "gate_up":
            fn = lambda: ops.pgemm_swiglu(aq, as_, wq, ws)  # noqa: E731
        elif name in ("o", "down"):
            fn = lambda: ops.pgemm_resid(aq, as_, wq, ws, resid)  # noqa: E731
        line(name, "mxfp8_fused", timed(fn, a.iters), N, K)
        line(name, "mxfp8_plain", timed(lambda: ops.pgemm(aq, as_, wq, ws), a.iters), N, K)
        try:
            xa = x[name].to(torch.float8_e4m3fn)
            wb = w[name].to(torch.float8_e4m3fn)
            one = torch.ones((), device=dev)
            line(name, "fp8_scaled_mm", timed(lambda: torch._scaled_mm(xa, wb.t(), scale_a=one, scale_b=one,
                                                                     out_dtype=torch.bfloat16), a.iters), N, K)
        except Exception as e:  # not in every torch build
            print(json.dumps({"proj": name, "impl": "fp8_scaled_mm", "error": str(e)[:200]}), flush=True)
    tot = {impl: sum(v.get(impl, 0) for v in out.values()) for impl in ("bf16_hipblaslt", "mxfp8_fused")}
    print(json.dumps({"rows": M, "bk": a.bk or 128, "waves": a.waves or 4, "group": a.group or 8, "areg": a.areg, "layer_us": {k: round(v, 1) for k, v in tot.items()},
                      "speedup": round(tot["bf16_hipblaslt"] / tot["mxfp8_fused"], 3)}), flush=True)
    # decode-step shapes: the bf16 weight-streaming GEMMs (wgemm.hip, fused
    # reductions) against the MX fp8 ones (wmx_kernel + the same reductions)
    for Md in a.decode_rows:
        ws_b = hip.wgemm_workspace(Md, max(c.qkv_dim, H), dev)
        ws_m = torch.empty(16 * Md * max(c.qkv_dim, H, I), dtype=torch.float32, device=dev)
        xd = {k: v[:Md].contiguous() for k, v in x.items()}
        md = {k: ops.mx_quant(v) for k, v in xd.items()}
        rd = bf(Md, H)
        nw = torch.ones(H, dtype=torch.bfloat16, device=dev)
        posd, slotd = pos[:Md].contiguous(), slot[:Md].contiguous()
        res = {}
        res["qkv"] = (timed_graph(lambda: hip.wgemm_rope_kv(xd["qkv"], w["qkv"], posd, slotd, cos_sin, kc, vc, c.n_heads,
                                                      ws_b), a.iters),
                      timed_graph(lambda: hip.wgemm_mx_rope_kv(*md["qkv"], *w8["qkv"], posd, slotd, cos_sin, kc, vc,
                                                         c.n_heads, ws_m), a.iters))
        res["o"] = (timed_graph(lambda: hip.wgemm_resid_norm(xd["o"], w["o"], rd, nw, 1e-5, ws_b), a.iters),
                    timed_graph(lambda: hip.wgemm_mx_resid_norm(*md["o"], *w8["o"], rd, nw, 1e-5, ws_m), a.iters))
        res["gate_up"] = (timed_graph(lambda: hip.wgemm_swiglu(xd["gate_up"], w["gate_up"]), a.iters),
                          timed_graph(lambda: hip.wgemm_mx_swiglu(*md["gate_up"], *w8["gate_up"]), a.iters))
        res["down"] = (timed_graph(lambda: hip.wgemm_resid_norm(xd["down"], w["down"], rd, nw, 1e-5, ws_b), a.iters),
                       timed_graph(lambda: hip.wgemm_mx_resid_norm(*md["down"], *w8["down"], rd, nw, 1e-5, ws_m), a.iters))
        for k, (tb, tm) in res.items():
            N, K = shapes[k]
            print(json.dumps({"decode_rows": Md, "proj": k, "bf16_wgemm_us": round(tb, 1), "mx_fp8_us": round(tm, 1),
                              "mx_weight_TBps": round(N * K / tm / 1e6, 2)}), flush=True)
        tb, tm = sum(v[0] for v in res.values()), sum(v[1] for v in res.values())
        print(json.dumps({"decode_rows": Md, "layer_us": {"bf16_wgemm": round(tb, 1), "mx_fp8": round(tm, 1)},
                          "speedup": round(tb / tm, 3)}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
