#!/usr/bin/env python3
"""Headline benchmark: classes indexed per second (BASELINE.json fallback metric).

One *step* = one complete ``analyze_project`` of a synthetic Spring Boot
monorepo through the production pipeline: snapshot of the branch head (git
objects read in place: ``ls-tree`` + native parallel inflate of every source
blob) -> native C++ parse of the in-memory tree -> graph build -> Phase 1
persist (SQLite, one transaction replacing the previous analysis, written by
a native thread) -> graph JSON -> cache publish.  Every step re-reads and
re-parses every file; nothing is cached across steps.  Enrichment
is disabled by default (BASELINE: "Indexing throughput with enrichment
disabled"); ``--enrich fake|local`` adds Phase 2/3 (``local`` = the optional
MI355X model, see dmcp/enrich/local.py).

Multi-GPU contract: launched by ``torch.distributed.run`` with one rank per
GPU; every rank indexes its own repository (weak scaling), the timed region
is bracketed by barrier + ``torch.cuda.synchronize()``, the MAX elapsed over
ranks is taken (all-reduce over RCCL when GPUs are present, gloo otherwise)
and rank 0 prints one JSON line with the whole-job aggregate.
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import shutil
import statistics
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "classes indexed/sec"
BASELINE_VALUE = None  # the reference publishes no throughput number


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--classes", type=int, default=2000, help="classes per synthetic repo (per rank)")
    ap.add_argument("--threads", type=int, default=0, help="parser threads per rank (0 = auto)")
    ap.add_argument("--enrich", default="none", choices=["none", "fake", "local"])
    ap.add_argument("--queries", type=int, default=200, help="graph_query / stack-trace latency samples")
    ap.add_argument("--workdir", default=None)
    return ap.parse_args(argv)


def main(argv=None) -> int:
    args = parse_args(argv)
    from dmcp.parallel.dist import init_from_env
    ctx = init_from_env()
    rank, world = ctx.rank, ctx.world
    logging.basicConfig(level=logging.WARNING, stream=sys.stderr)
    from dmcp.app import App
    from dmcp.config import Config
    from dmcp.utils import synth
    from dmcp.utils.tracing import METRICS

    try:
        cpus = len(os.sched_getaffinity(0))  # the CPUs this process may run on (cgroup / cpuset aware)
    except (AttributeError, OSError):
        cpus = os.cpu_count() or 8
    # 8 parser threads: the analysis is bound by its SQLite writer thread, 8 = 16 = 32 threads on one
    # MI355X host (profiles/bench_r2_threads_ab.txt), and fewer leave CPUs to the other ranks
    threads = args.threads or max(1, min(8, cpus // max(1, ctx.local_world)))
    work = args.workdir or tempfile.mkdtemp(prefix=f"dmcp-bench-r{rank}-")
    repo = os.path.join(work, f"shop{rank}")
    fqcns = synth.java_spring_repo(repo, n_classes=args.classes, base_package=f"co.acme.shop{rank}", seed=rank + 1)
    cfg = Config(db_path=os.path.join(work, "bench.db"), git_clone_base_path=os.path.join(work, "clones"),
                 parser_threads=threads, enrich_backend=args.enrich if args.enrich != "none" else "null",
                 require_enrichment_for_analyze=False, recover_stuck_on_start=False)
    app = App(cfg)
    try:
        n_classes = 0
        stats_acc = {}
        for _ in range(args.warmup):
            app.indexer.analyze_project(repo)
        ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            r = app.indexer.analyze_project(repo)
            n_classes += r.classes_analyzed
            for k, v in r.stats.items():
                if k.startswith("analyze."):
                    stats_acc[k] = stats_acc.get(k, 0.0) + v
        ctx.synchronize()
        elapsed = time.perf_counter() - t0
        # whole-job aggregate: MAX elapsed over ranks, SUM of classes
        elapsed = ctx.max(elapsed)[0]
        total_classes = int(ctx.sum(float(n_classes))[0])
        # query latencies on the indexed graph (BASELINE configs 3/4)
        extra = {"phaseMsPerStep": {k: round(v / max(1, args.steps), 2) for k, v in stats_acc.items()},
                 "classesPerRepo": r.classes_analyzed, "parserThreadsPerRank": threads}
        if rank == 0 and args.queries > 0:
            project = f"shop{rank}"
            qs = [f"{project}:endpoints", f"{project}:classes", f"{project}:OrderService:methods:+logic",
                  f"{project}:UserController:dependencies", f"{project}:entrypoints:+logic",
                  f"{project}:PaymentService:?list"]
            lat = []
            for i in range(args.queries):
                q0 = time.perf_counter()
                app.graph_query.query(qs[i % len(qs)])
                lat.append((time.perf_counter() - q0) * 1e3)
            st_lat = []
            trace = synth.stack_trace_for(fqcns, 20)
            for _ in range(max(10, args.queries // 10)):
                q0 = time.perf_counter()
                app.context.get_stack_trace_context(trace)
                st_lat.append((time.perf_counter() - q0) * 1e3)
            lat.sort()
            st_lat.sort()
            extra["graphQueryMs"] = {"p50": round(lat[len(lat) // 2], 3), "p99": round(lat[int(len(lat) * 0.99) - 1], 3)}
            extra["stackTrace20Ms"] = {"p50": round(st_lat[len(st_lat) // 2], 3),
                                       "p99": round(st_lat[max(0, int(len(st_lat) * 0.99) - 1)], 3)}
        value = total_classes / elapsed if elapsed > 0 else 0.0
        ms_per_step = elapsed / max(1, args.steps) * 1e3
        if rank == 0:
            line = {"metric": METRIC, "value": round(value, 2), "unit": "classes/s", "n_gpus": world,
                    "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
                    "higher_is_better": True, "scaling": "weak",
                    "vs_baseline": (round(value / BASELINE_VALUE, 4) if BASELINE_VALUE else None),
                    "dtype": "n/a (CPU text indexing)", "data": "synthetic (generated Spring Boot monorepo, "
                    "local git repo, random-free deterministic)",
                    "config": {"model": f"synthetic-java-spring-monorepo-{args.classes}-classes",
                               "global_batch": args.classes * world, "seq_len": None,
                               "parallelism": f"dp{world} (one repo per rank)",
                               "enrichment": args.enrich},
                    "extra": extra}
            print(json.dumps(line), flush=True)
    finally:
        app.close()
        if args.workdir is None:
            shutil.rmtree(work, ignore_errors=True)
        ctx.shutdown()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
