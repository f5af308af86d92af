#!/usr/bin/env python3
"""Decode-step microbenchmark of the local enrichment model (GPU box).

Reproduces the steady state of ``bench_enrich.py`` without the grammar
engine: ``--batch`` sequences that share a ``--prefix``-token prompt prefix
(instructions + README) and each own ``--ctx`` more tokens of context, plus
``--extra`` jump-forward rows (consecutive positions of the first slots), so
one step runs ``batch + extra`` rows through the captured decode graph.

Reports, per step: device time of back-to-back graph replays (no host work
between them), and the engine-like loop time (pack inputs, replay, copy the
selected ids back, convert to a list).  With ``--fused 0/1`` the decode GEMMs
run on hipBLASLt or on the fused gfx950 kernels (dmcp.ops.fused).

    python scripts/bench_step.py --fused 1
    rocprofv3 --kernel-trace --stats -d gpurun_out/step -o step -- python3 scripts/bench_step.py
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="dmcp-coder-1b")
    ap.add_argument("--kv-dtype", default="bf16", choices=["bf16", "fp8"],
                    help="KV cache storage (fp8 = e4m3, half the attention bytes)")
    ap.add_argument("--decode-dtype", default="bf16", choices=["bf16", "fp8"],
                    help="decode projections: bf16 or fp8 weights x MXFP8 activations")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--extra", type=int, default=14)
    ap.add_argument("--prefix", type=int, default=4151)
    ap.add_argument("--ctx", type=int, default=2500)
    ap.add_argument("--max-seq", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--fused", type=int, default=-1, help="-1 = model default, 0 = hipBLASLt, 1 = fused kernels")
    ap.add_argument("--wgemm", type=int, default=-1, help="-1 = model default, 0 = hipBLASLt for > 16 rows")
    ap.add_argument("--tghead", type=int, default=-1, help="0 = the weight-streaming LM head at every row count")
    ap.add_argument("--tgemm", type=int, default=-1,
                    help="-1 = model default, 0 = hipBLASLt (projections + LM head) for > 512 rows")
    ap.add_argument("--wgemm-aux", type=int, default=0, choices=[0, 2],
                    help="cache policy of the weight-streaming GEMM's weight loads (2 = nt)")
    ap.add_argument("--jitter", type=float, default=0.0,
                    help="per-sequence own length uniform in ctx x [1 - j, 1 + j] (the engine's mix of progress)")
    ap.add_argument("--adjacent", action="store_true",
                    help="jump rows next to their sequence's row (the engine's row order) instead of at the end")
    a = ap.parse_args(argv)

    from dmcp.enrich.local import LocalEngine
    from dmcp.models.llm import LocalLM, preset
    from dmcp.ops import hip


    torch.cuda.set_device(0)
    cfg = preset(a.preset, max_batch=a.batch, max_seq=a.max_seq, kv_dtype=a.kv_dtype)
    cfg = preset(a.preset, max_batch=a.batch, max_seq=a.max_seq, kv_dtype=a.kv_dtype, decode_dtype=a.decode_dtype,
                 max_rows=max(cfg.max_rows, a.batch + a.extra))
    model = LocalLM(cfg, device="cuda:0")
    if a.fused >= 0:
        model.use_fused = bool(a.fused)
        model.fused_max_rows = 128 if a.fused else 0
    if a.wgemm >= 0:
        model.use_wgemm = bool(a.wgemm)
    if a.tgemm == 0:
        model.use_tgemm = False
        model.tg_head = False
    if a.tghead == 0:
        model.tg_head = False
    hip.wgemm_set_aux(a.wgemm_aux)
    eng = LocalEngine(model)
    g = torch.Generator().manual_seed(0)
    if a.prefix:
        model.set_prefix(torch.randint(0, 256, (a.prefix,), generator=g).tolist())
    n = a.batch + a.extra
    toks = torch.randint(0, 256, (n,), generator=g).tolist()
    u = (torch.rand(a.batch, generator=g) * 2 - 1).tolist()
    ctxs = [max(1, int(round(a.ctx * (1 + a.jitter * x)))) for x in u]
    slots = list(range(a.batch)) + [i % a.batch for i in range(a.extra)]
    poss = [a.prefix + ctxs[sl] + (i // a.batch) for i, sl in enumerate(slots)]
    if a.adjacent:  # each sequence's jump rows right after its own row
        order = sorted(range(n), key=lambda i: (slots[i], i))
        slots, poss = [slots[i] for i in order], [poss[i] for i in order]
    mrows = [0] * n
    graphs = eng.graphs
    for _ in range(3):
        graphs.run(toks, slots, poss, mrows)[1].cpu()
    torch.cuda.synchronize()
    # device time: back-to-back replays (and the host time inside each
    # run() call: the CPU cost of packing + H2D + hipGraphLaunch)
    t0 = time.perf_counter()
    cpu = 0.0
    for _ in range(a.iters):
        c0 = time.perf_counter()
        graphs.run(toks, slots, poss, mrows)
        cpu += time.perf_counter() - c0
    torch.cuda.synchronize()
    dev_ms = (time.perf_counter() - t0) / a.iters * 1e3
    launch_ms = cpu / a.iters * 1e3
    # the engine's pipelined loop: launch step k, then wait for step k-1's ids
    host = [torch.zeros(n, dtype=torch.int32).pin_memory() for _ in range(2)]
    prev = None
    t0 = time.perf_counter()
    for it in range(a.iters):
        _, ids = graphs.run(toks, slots, poss, mrows)
        host[it % 2].copy_(ids, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        if prev is not None:
            prev.synchronize()
        prev = ev
    prev.synchronize()
    pipe_ms = (time.perf_counter() - t0) / a.iters * 1e3
    # engine-like loop: wait for the ids and convert them every step
    t0 = time.perf_counter()
    for _ in range(a.iters):
        graphs.run(toks, slots, poss, mrows)[1].cpu().tolist()
    loop_ms = (time.perf_counter() - t0) / a.iters * 1e3
    kv_bytes = 2 * cfg.layers * cfg.n_kv_heads * cfg.head_dim * cfg.kv_elem_bytes * (sum(ctxs) + a.batch + a.prefix)
    w_bytes = 2 * (cfg.param_count() - cfg.vocab_size * cfg.hidden)
    print(json.dumps({"bench": "decode_step", "preset": a.preset, "kv_dtype": a.kv_dtype, "decode_dtype": a.decode_dtype, "rows": n, "batch": a.batch, "prefix": a.prefix,
                      "ctx": a.ctx, "jitter": a.jitter, "adjacent": a.adjacent, "fused": bool(getattr(model, "use_fused", False)),
                      "tgemm": bool(getattr(model, "use_tgemm", False)),
                      "tg_head": bool(getattr(model, "tg_head", False)), "wgemm_aux": a.wgemm_aux,
                      "prefix_splits": hip.prefix_mfma_splits(a.batch + a.extra, cfg.n_heads // cfg.n_kv_heads,
                                                              cfg.n_kv_heads),
                      "device_ms": round(dev_ms, 3), "loop_ms": round(loop_ms, 3),
                      "launch_cpu_ms": round(launch_ms, 3), "pipelined_ms": round(pipe_ms, 3),
                      "host_gap_ms": round(loop_ms - dev_ms, 3),
                      "sol_ms_at_6p3TBps": round((kv_bytes + w_bytes) / 6.3e12 * 1e3, 3),
                      "weight_MB": round(w_bytes / 1e6, 1), "kv_MB": round(kv_bytes / 1e6, 1)}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
