#!/usr/bin/env python3
"""Per-class prefill of the local enrichment model (GPU box): one sequence's
own prompt (``--tokens``) after a shared prefix (``--prefix``), as the engine
admits classes.  Prints ms per prefill and prompt tokens/s.

    rocprofv3 --kernel-trace --stats -d gpurun_out/pf -o pf -- python3 scripts/bench_prefill.py
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="dmcp-coder-1b")
    ap.add_argument("--prefix", type=int, default=4151)
    ap.add_argument("--tokens", type=int, default=2100)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from dmcp.models.llm import LocalLM, preset
    model = LocalLM(preset(a.preset, max_batch=8, max_seq=8192), device="cuda:0")
    g = torch.Generator().manual_seed(0)
    if a.prefix:
        model.set_prefix(torch.randint(0, 256, (a.prefix,), generator=g).tolist())
    toks = torch.randint(0, 256, (a.tokens,), generator=g, dtype=torch.int32)
    for _ in range(3):
        start = model.fork_prefix(0)
        model.forward_tokens(toks, 0, start)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.iters):
        start = model.fork_prefix(i % 8)
        model.forward_tokens(toks, i % 8, start)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / a.iters * 1e3
    cfg = model.cfg
    flops = 2 * a.tokens * (cfg.param_count() - 2 * cfg.vocab_size * cfg.hidden) + \
        4 * cfg.layers * cfg.n_heads * cfg.head_dim * a.tokens * (a.prefix + a.tokens / 2)
    print(json.dumps({"bench": "prefill", "prefix": a.prefix, "tokens": a.tokens, "ms": round(ms, 3),
                      "tokens_per_s": round(a.tokens / ms * 1e3, 1), "TFLOPs": round(flops / ms / 1e9, 1)}),
          flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
