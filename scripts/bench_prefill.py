#!/usr/bin/env python3
"""Prefill of the local enrichment model (GPU box), as the engine admits
classes: ``--seqs`` sequences of ``--tokens`` own prompt tokens after a shared
prefix of ``--prefix`` tokens, in ONE ``LocalLM.prefill_batch`` (packed GEMMs
+ varlen attention) -- or ``--seqs 1`` for the single-sequence path.  Prints
ms per batch, ms per class and prompt tokens/s (fp8 or bf16 KV cache).

    rocprofv3 --kernel-trace --stats -d gpurun_out/pf -o pf -- python3 scripts/bench_prefill.py --seqs 12
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
    ap.add_argument("--seqs", type=int, default=12)
    ap.add_argument("--kv-dtype", default="fp8", choices=["bf16", "fp8"])
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--prefill-dtype", default="bf16", choices=["auto", "bf16", "fp8"])
    a = ap.parse_args()
    from dmcp.models.llm import LocalLM, preset
    model = LocalLM(preset(a.preset, max_batch=max(8, a.seqs), max_seq=8192, kv_dtype=a.kv_dtype,
                           prefill_dtype=a.prefill_dtype), device="cuda:0")
    g = torch.Generator().manual_seed(0)
    P = 0
    if a.prefix:
        P = model.set_prefix(torch.randint(0, 256, (a.prefix,), generator=g).tolist())
    toks = torch.randint(0, 256, (a.tokens,), generator=g, dtype=torch.int32).tolist()

    def one_batch():
        for s in range(a.seqs):
            model.fork_prefix(s)
        return model.prefill_batch([(toks, s, P) for s in range(a.seqs)])
    for _ in range(2):
        one_batch()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        one_batch()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / a.iters * 1e3
    flops = 2 * model.cfg.param_count() * a.tokens * a.seqs
    print(json.dumps({"bench": "prefill_batch", "seqs": a.seqs, "tokens": a.tokens, "prefix": P,
                      "kv_dtype": a.kv_dtype, "prefill_dtype": a.prefill_dtype, "ms_per_batch": round(ms, 3), "ms_per_class": round(ms / a.seqs, 3),
                      "prompt_tokens_per_s": round(a.tokens * a.seqs / ms * 1e3, 1),
                      "weight_tflops": round(flops / ms / 1e9, 1)}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
