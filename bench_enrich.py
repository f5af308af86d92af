#!/usr/bin/env python3
"""GPU benchmark of the local enrichment backend (MI355X extension).

Measures classes enriched per second, generated tokens per second and the
batched decode step time of :class:`dmcp.enrich.local.LocalEngine` on synthetic
classes of a generated Spring repository (random-init weights of the named
preset; no checkpoint is available offline).  With ``torch.distributed.run``
each rank is an independent replica on its own GPU (data parallel, no
collectives in the hot path); rank 0 prints one JSON line with the whole-job
aggregate (MAX elapsed over ranks, all-reduced over RCCL).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="dmcp-coder-1b")
    ap.add_argument("--kv-dtype", default="fp8", choices=["bf16", "fp8"],
                    help="KV cache storage (fp8 = e4m3, half the attention bytes)")
    ap.add_argument("--prefill-dtype", default="auto", choices=["auto", "bf16", "fp8"],
                    help="batched-prefill projections: bf16 (hipBLASLt) or fp8 (MXFP8 kernels, csrc/pgemm.hip)")
    ap.add_argument("--decode-dtype", default="bf16", choices=["bf16", "fp8"],
                    help="decode-step projections: bf16, or fp8 weights x MXFP8 activations (csrc/pgemm.hip)")
    ap.add_argument("--classes", type=int, default=1024, help="classes per rank")
    ap.add_argument("--batch", type=int, default=768, help="concurrent sequences (KV slots)")
    ap.add_argument("--max-seq", type=int, default=8192)
    ap.add_argument("--max-rows", type=int, default=0,
                    help="rows per decode step incl. jump-forward rows (0 = 1.5 x batch, >= 256)")
    ap.add_argument("--prompt-chars", type=int, default=2048)
    ap.add_argument("--readme-chars", type=int, default=4000,
                    help="project README in every prompt (the reference sends up to 10,000 chars)")
    ap.add_argument("--no-shared-prefix", action="store_true",
                    help="prefill and attend to the instructions + README per class instead of once")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--no-jump", action="store_true", help="disable jump-forward over forced tokens")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="synchronous engine loop (host waits for every step's ids before building the next)")
    ap.add_argument("--admit-min", type=int, default=0,
                    help="free KV slots before a running batch admits new classes (0 = engine default, batch/16)")
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--max-new-tokens", type=int, default=4096, help="reply budget (LOCAL_LLM_MAX_NEW_TOKENS)")
    ap.add_argument("--no-fork", action="store_true", help="methods decoded in sequence, not as branches")
    ap.add_argument("--reply-shape", default="derived", choices=["derived", "legacy"],
                    help="string caps / steps of the replies: derived from the reply budget (the service default, "
                         "256 / 128 / 64 bytes, 4 steps at 4,096 tokens) or the round-4 fixed 96 / 64 / 40, 3")
    ap.add_argument("--checkpoint", default="",
                    help="a Llama-format checkpoint directory (LOCAL_LLM_MODEL_PATH) instead of the preset's random "
                         "weights; with --write-checkpoint a synthetic one (trained-like random weights, Llama-3.2-1B "
                         "geometry, the code BPE) is written there first when it has no config.json")
    ap.add_argument("--write-checkpoint", action="store_true")
    ap.add_argument("--fork-max-context", type=int, default=-1,
                    help="fork only classes with at most this many own prompt tokens (-1: the engine default)")
    args = ap.parse_args(argv)

    import torch
    from dmcp.enrich.local import LocalEngine, ReplyShape
    from dmcp.enrich.types import EnrichmentInput
    from dmcp.models.llm import LocalLM, preset

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl")
    max_rows = args.max_rows or max(args.batch, min(1024, max(256, args.batch + args.batch // 2)))
    if args.checkpoint:
        from dmcp.enrich.tokenizer import load_local_model
        if args.write_checkpoint and not os.path.exists(os.path.join(args.checkpoint, "config.json")):
            from dmcp.utils import synth
            if rank == 0:
                synth.llama_checkpoint(args.checkpoint, device=f"cuda:{local}")
            if dist is not None:
                dist.barrier()
        model, tok = load_local_model(args.checkpoint, device=f"cuda:{local}", max_batch=args.batch,
                                      max_seq=args.max_seq, kv_dtype=args.kv_dtype, prefill_dtype=args.prefill_dtype,
                                      decode_dtype=args.decode_dtype, max_rows=max_rows)
        cfg = model.cfg
    else:
        cfg = preset(args.preset, max_batch=args.batch, max_seq=args.max_seq, kv_dtype=args.kv_dtype,
                     prefill_dtype=args.prefill_dtype, decode_dtype=args.decode_dtype, max_rows=max_rows)
        model = LocalLM(cfg, device=f"cuda:{local}", seed=rank)
        tok = None
        if cfg.tokenizer:
            from dmcp.enrich.tokenizer import load_asset_tokenizer
            tok = load_asset_tokenizer(cfg.tokenizer)
    eng = LocalEngine(model, use_graphs=not args.no_graphs, jump_forward=not args.no_jump,
                      shared_prefix=not args.no_shared_prefix, pipeline=not args.no_pipeline,
                      admit_min=args.admit_min or None, tokenizer=tok, max_new_tokens=args.max_new_tokens,
                      fork_methods=not args.no_fork,
                      reply_shape=ReplyShape.LEGACY if args.reply_shape == "legacy" else None,
                      **({} if args.fork_max_context < 0 else {"fork_max_context": args.fork_max_context}))
    para = ("The shop platform sells products to retail customers. Orders move from CART to PAID to "
            "SHIPPED; payments are captured through the payment gateway and refunds are issued by the "
            "back office. Inventory is reserved when an order is paid and released on cancellation.\n\n")
    readme = "# Acme Shop\n\n"
    while len(readme) < args.readme_chars:
        readme += para
    readme = readme[:args.readme_chars] if args.readme_chars > 0 else "Synthetic commerce platform"
    body = ("    public OrderResponse create(OrderRequest request) {\n"
            "        Order order = repository.save(Order.from(request));\n"
            "        events.publish(new OrderCreated(order.id()));\n        return OrderResponse.of(order);\n    }\n")

    def make(i: int) -> EnrichmentInput:
        src = f"package co.acme.shop.d{i % 30};\n\n@Service\npublic class Svc{i} {{\n"
        while len(src) < args.prompt_chars:
            src += body
        return EnrichmentInput(src + "}\n", f"co.acme.shop.d{i % 30}.Svc{i}", "java", "SERVICE",
                               ["create", "update", "find", "delete", "list", "validate"][: 2 + i % 5])

    inputs = [make(rank * 100000 + i) for i in range(args.classes)]
    eng.generate([make(-1 - i) for i in range(args.warmup)], readme)
    for k in eng.stats:
        eng.stats[k] = 0
    if eng.graphs is not None:
        eng.graphs.timing = {k: 0.0 for k in eng.graphs.timing}
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    outs = eng.generate(inputs, readme)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ok = sum(1 for o in outs if o.startswith('{"description"'))
    st = dict(eng.stats)
    tot = torch.tensor([elapsed, float(ok), st["generated_tokens"], st["prompt_tokens"]], dtype=torch.float64,
                       device="cuda")
    if dist is not None:
        mx = tot[:1].clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        tot[0] = mx[0]
    elapsed, ok_all, gen_all, prompt_all = (float(x) for x in tot.tolist())
    if rank == 0:
        print(json.dumps({
            "metric": "classes enriched/sec (local MI355X model)", "value": round(ok_all / elapsed, 3),
            "unit": "classes/s", "n_gpus": world, "higher_is_better": True, "scaling": "weak",
            "dtype": "bf16", "data": "synthetic classes, " + ("checkpoint " + args.checkpoint if args.checkpoint
                                                               else "random-init weights"),
            "config": {"model": cfg.name, "params_b": round(cfg.param_count() / 1e9, 3), "batch": args.batch,
                       "max_rows": cfg.max_rows, "kv_dtype": cfg.kv_dtype, "prefill_dtype": "fp8" if model.prefill_fp8 else "bf16", "decode_dtype": cfg.decode_dtype,
                       "max_seq": args.max_seq, "prompt_chars": args.prompt_chars,
                       "readme_chars": args.readme_chars, "graphs": not args.no_graphs, "reply_shape": [eng.reply_shape.desc, eng.reply_shape.method, eng.reply_shape.step,
                                                                          eng.reply_shape.max_steps],
                       "jump_forward": not args.no_jump, "shared_prefix": not args.no_shared_prefix,
                       "pipeline": not args.no_pipeline},
            "shared_prefix_tokens": st["prefix_tokens"], "prefix_ms": round(1e3 * st["prefix_s"], 3),
            "generated_tokens_per_s": round(gen_all / elapsed, 1),
            "prompt_tokens_per_s": round(prompt_all / elapsed, 1),
            "decode_step_ms": round(1e3 * st["decode_s"] / max(1, st["decode_steps"]), 3),
            "prefill_ms_avg": round(1e3 * st["prefill_s"] / max(1, st["prefills"]), 3),
            "prefill_s": round(st["prefill_s"], 3), "prefill_gpu_s": round(st.get("prefill_gpu_s", 0.0), 3),
            "prefill_batches": st["prefill_batches"],
            "decode_s": round(st["decode_s"], 3), "host_ms_per_step": round(1e3 * st["host_s"] / max(1, st["decode_steps"]), 3),
            "launch_ms_per_step": round(1e3 * st.get("launch_s", 0) / max(1, st["decode_steps"]), 3),
            "wait_ms_per_step": round(1e3 * st.get("wait_s", 0) / max(1, st["decode_steps"]), 3),
            "graph_timing_ms_per_step": ({k: round(1e3 * v / max(1, st["decode_steps"]), 3)
                                          for k, v in eng.graphs.timing.items()} if eng.graphs else None),
            "forks": st.get("forks", 0), "fork_branches": st.get("fork_branches", 0),
            "admit_min": eng.admit_min,
            "decode_steps": st["decode_steps"], "rows_per_step": round(st["decode_rows"] / max(1, st["decode_steps"]), 1),
            "elapsed_s": round(elapsed, 3), "classes": int(ok_all),
            "prompt_tokens_per_class": round(st["prompt_tokens"] / max(1, st["prefills"]), 1),
            "generated_tokens_per_class": round(st["generated_tokens"] / max(1, ok_all), 1),
            "choice_waits": st.get("choice_waits", 0), "type_corrections": st.get("type_corrections", 0),
            # the timed session's slowest loop iterations: (ms, host ms by phase)
            "slowest_iters": getattr(eng, "slow_iters", None)}),
            flush=True)
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
