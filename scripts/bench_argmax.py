"""masked_argmax timing (dmcp_kernels.hip: masked_argmax_kernel): the engine's
prefill selection over [rows, 128,256] bf16 logits under a grammar mask
table.  One JSON line per row count; DMCP_HIPOPS_SO=<other build> times
another library (A/B).

  python scripts/bench_argmax.py [--rows 16 64 128 256] [--vocab 128256]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, nargs="+", default=[16, 64, 128, 256])
    ap.add_argument("--vocab", type=int, default=128256)
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    import torch
    from dmcp.ops import hip, reference
    V = args.vocab
    W = (V + 31) // 32
    g = torch.Generator(device="cuda").manual_seed(0)
    masks = torch.randint(-2 ** 31, 2 ** 31 - 1, (8, W), device="cuda", dtype=torch.int32, generator=g)
    for B in args.rows:
        logits = torch.randn(B, V, device="cuda", generator=g).to(torch.bfloat16)
        midx = torch.randint(0, 8, (B,), device="cuda", dtype=torch.int32, generator=g)
        got = hip.masked_argmax(logits, masks, vocab=V, mask_idx=midx)
        ok = bool(torch.equal(got, reference.masked_argmax(logits, masks, vocab=V, mask_idx=midx)))
        for _ in range(5):
            hip.masked_argmax(logits, masks, vocab=V, mask_idx=midx, out=got)
        # captured in a graph: timed back to back on the device, without the
        # Python wrapper's per-call host cost (~40 us, more than the kernel)
        graph = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            with torch.cuda.graph(graph, stream=side):
                for _ in range(args.reps):
                    hip.masked_argmax(logits, masks, vocab=V, mask_idx=midx, out=got)
        torch.cuda.current_stream().wait_stream(side)
        graph.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        graph.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / args.reps
        print(json.dumps({"bench": "masked_argmax", "lib": os.environ.get("DMCP_HIPOPS_SO") or "in-tree",
                          "rows": B, "vocab": V, "us": round(us, 2), "GBps": round(B * V * 2 / us / 1e3, 1),
                          "matches_fp32_reference": ok}), flush=True)


if __name__ == "__main__":
    main()
