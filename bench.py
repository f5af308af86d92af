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
disabled"); ``--enrich fake`` adds Phase 2/3 with the offline fake backend.

``extra.enrichLocal`` (GPU present, ``--enrich-local-classes`` > 0): after
the headline, each rank runs a real ``analyze_project`` of a
``--enrich-local-classes``-class repository with the optional MI355X
enrichment backend in the service configuration -- one worker process per
GPU (dmcp/enrich/workers.py, spawned before this process touches HIP),
every pending class streamed to it, fp8 KV cache, 512 concurrent sequences
-- and reports classes enriched per second through the whole pipeline plus
the engine's per-step device / host split.  It runs once per preset of
``--enrich-local-presets``: ``dmcp-coder-1b`` (byte vocabulary) ->
``extra.enrichLocal``; ``llama3.2-1b-code`` (Llama-3.2-1B shapes, 128,256-id
code BPE: a real 1B code model's operating point) -> ``extra.enrichLocalLlama``.

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
    ap.add_argument("--enrich-local-classes", type=int, default=256,
                    help="classes of the end-to-end local-model enrichment run (extra.enrichLocal; 0 = skip)")
    ap.add_argument("--enrich-local-kv", default="fp8", choices=["bf16", "fp8"])
    ap.add_argument("--enrich-local-prefill", default="auto", choices=["auto", "bf16", "fp8"],
                    help="batched-prefill GEMMs of the enrichment worker (auto = MXFP8 on gfx950)")
    ap.add_argument("--enrich-local-batch", type=int, default=768)
    ap.add_argument("--enrich-local-presets", default="dmcp-coder-1b,llama3.2-1b-code")
    ap.add_argument("--remote-steps", type=int, default=3,
                    help="timed analyses on the remote-repository path (extra.remotePath; 0 = skip)")
    ap.add_argument("--lang-files", type=int, default=1000,
                    help="source files of the TS / Go indexing runs (extra.tsIndex / extra.goIndex; 0 = skip)")
    ap.add_argument("--lang-steps", type=int, default=5)
    ap.add_argument("--pool-classes", type=int, default=257,
                    help="classes of extra.enrichLocalPool: ONE project dealt by ONE GpuWorkerPool over --gpus GPUs "
                         "(the service's production layout, strong scaling; 0 = skip)")
    ap.add_argument("--pool-preset", default="llama3.2-1b-code")
    ap.add_argument("--small-project-classes", type=int, default=33,
                    help="classes of the latency-bound enrichment run (extra.enrichLocal*.smallProject: what "
                         "each of 8 GPUs gets when one 257-class project is dealt over 8; 0 = skip)")
    return ap.parse_args(argv)


EXTRA_KEYS = {"dmcp-coder-1b": "enrichLocal", "llama3.2-1b-code": "enrichLocalLlama"}
POOL_KEY = "__pool__"


def _spawn_enrich_pools(args):
    """One enrichment worker per preset for this rank's GPU, spawned BEFORE
    this process initialises HIP (each child stays idle -- no torch import --
    until its init; they run one after the other, each closed after its run)."""
    if args.enrich_local_classes <= 0:
        return {}
    try:
        import torch
        if torch.cuda.device_count() <= 0:  # counts devices without creating a HIP context
            return {}
        from dmcp.enrich.workers import GpuWorkerPool
        local = int(os.environ.get("LOCAL_RANK", "0"))
        mb = args.enrich_local_batch
        pools = {}
        for name in [p.strip() for p in args.enrich_local_presets.split(",") if p.strip()]:
            model = {"preset": name, "kv_dtype": args.enrich_local_kv, "prefill_dtype": args.enrich_local_prefill,
                     "max_batch": mb,
                     "max_rows": max(mb, min(1024, max(256, mb * 3 // 2))), "seed": 0}
            pools[name] = GpuWorkerPool([f"cuda:{local}"], model, engine={"max_new_tokens": 4096}, init=False,
                                        start_timeout_s=600)
        if args.pool_classes > 0 and int(os.environ.get("RANK", "0")) == 0:
            # extra.enrichLocalPool: rank 0's service-style pool, one worker per
            # GPU of the job (idle children until its turn, after the per-rank runs)
            n = max(1, min(args.gpus, torch.cuda.device_count()))
            model = {"preset": args.pool_preset, "kv_dtype": args.enrich_local_kv,
                     "prefill_dtype": args.enrich_local_prefill, "max_batch": mb,
                     "max_rows": max(mb, min(1024, max(256, mb * 3 // 2))), "seed": 0}
            pools[POOL_KEY] = GpuWorkerPool([f"cuda:{i}" for i in range(n)], model,
                                            engine={"max_new_tokens": 4096}, init=False, start_timeout_s=900)
        return pools
    except Exception as e:  # the headline does not depend on it
        logging.getLogger("bench").warning("enrichment worker not started: %s", e)
        return {}


def world_scale(ctx) -> float:
    """Ranks whose engine statistics the local stats stand for (every rank
    runs the same-sized project: whole-job token rate = local x world)."""
    return float(ctx.world)


def _enrich_local(pool, args, ctx, work, rank):
    """extra.enrichLocal: one warm-up analysis (hipGraph captures, allocator),
    then the timed analyze_project of a fresh repository, MAX over ranks."""
    from dmcp.app import App
    from dmcp.config import Config
    from dmcp.enrich.workers import ProcessLLMBackend
    from dmcp.utils import synth
    # every collective below is entered by every rank, whatever fails where
    # (a rank that raised before a barrier would leave the others waiting)
    t_init = time.perf_counter()
    err = None
    try:
        if pool is None:
            raise RuntimeError("no enrichment worker on this rank")
        pool.init()
    except Exception as e:
        err = e
    init_s = time.perf_counter() - t_init
    if ctx.sum(1.0 if err else 0.0)[0] > 0:
        raise RuntimeError(f"enrichment worker init failed on some rank: {err!r}")
    be = ProcessLLMBackend(pool)
    cfg = Config(db_path=os.path.join(work, "enrich.db"), git_clone_base_path=os.path.join(work, "eclones"),
                 require_enrichment_for_analyze=True, recover_stuck_on_start=False)
    app = App(cfg, backend=be)
    try:
        warm = os.path.join(work, f"warm{rank}")
        synth.java_spring_repo(warm, n_classes=min(64, max(8, args.enrich_local_classes // 4)),
                               base_package=f"co.acme.warm{rank}", seed=rank + 101)
        try:
            app.indexer.analyze_project(warm)
        except Exception as e:
            err = e
        if ctx.sum(1.0 if err else 0.0)[0] > 0:
            raise RuntimeError(f"enrichLocal warm-up failed on some rank: {err!r}")
        repo = os.path.join(work, f"enrich{rank}")
        synth.java_spring_repo(repo, n_classes=args.enrich_local_classes, base_package=f"co.acme.enr{rank}",
                               seed=rank + 201)
        for w in pool.workers:
            w.stats = {}
        ctx.barrier()
        t0 = time.perf_counter()
        try:
            r = app.indexer.analyze_project(repo)
        except Exception as e:
            r, err = None, e
        elapsed = time.perf_counter() - t0
        mx = ctx.max(elapsed)[0]
        bad = ctx.sum(1.0 if r is None else 0.0)[0]
        tot = ctx.sum(float(r.stats.get("enriched", 0)) if r else 0.0, float(r.classes_analyzed) if r else 0.0)
        if bad:
            raise RuntimeError(f"enrichLocal analysis failed on {int(bad)} rank(s): {err!r}")
        st = be.stats()
        steps = max(1.0, st.get("decode_steps", 0))
        small = None
        if args.small_project_classes > 0:
            # one small project alone on this GPU: the latency-bound tail each
            # GPU runs when a 257-class project is dealt over 8 (strong scaling)
            srepo = os.path.join(work, f"small{rank}")
            synth.java_spring_repo(srepo, n_classes=args.small_project_classes, base_package=f"co.acme.sml{rank}",
                                   seed=rank + 301)
            for w in pool.workers:  # a worker's stats are its last session's
                w.stats = {}
            ctx.barrier()
            t1 = time.perf_counter()
            try:
                rs = app.indexer.analyze_project(srepo)
            except Exception as e:
                rs, err = None, e
            smx = ctx.max(time.perf_counter() - t1)[0]
            if ctx.sum(1.0 if rs is None else 0.0)[0] == 0:
                ph2 = ctx.max(rs.stats.get("analyze.phase2", 0.0) / 1e3)[0]
                d = be.stats()
                ss = max(1.0, d.get("decode_steps", 0))
                # where a latency-bound run's time goes: steps x step time vs prefill and host
                small = {"classes": rs.classes_analyzed, "enriched": int(rs.stats.get("enriched", 0)),
                         "elapsedS": round(smx, 3), "phase2S": round(ph2, 3),
                         "classesPerSec": round(rs.classes_analyzed / smx, 2),
                         "decodeSteps": int(d.get("decode_steps", 0)),
                         "rowsPerStep": round(d.get("decode_rows", 0) / ss, 1),
                         "decodeStepMs": round(1e3 * d.get("decode_s", 0) / ss, 3),
                         "decodeS": round(d.get("decode_s", 0), 3),
                         "prefillGpuS": round(d.get("prefill_gpu_s", 0), 3),
                         "generatedTokensPerClass": round(d.get("generated_tokens", 0) / max(1, rs.classes_analyzed),
                                                          1)}
            else:
                small = {"error": repr(err)[:300]}
        wit = (pool.workers[0].info or {}).get("witness") if pool.workers else None
        return {"classesPerSec": round(tot[0] / mx, 2), "classesEnriched": int(tot[0]),
                "device": wit, "graphReplays": int(st.get("graph_replays", 0)),
                "graphKernelsPerStep": round(st.get("graph_kernels", 0) / max(1, st.get("graph_replays", 0)), 1),
                "smallProject": small,
                "promptTokensPerClass": round(st.get("prompt_tokens", 0) / max(1, st.get("prefills", 1)), 1),
                "generatedTokensPerClass": round(st.get("generated_tokens", 0) / max(1, tot[0]), 1),
                # shape-invariant: the reply caps grew this round (ReplyShape.from_budget)
                "generatedTokensPerSec": round(st.get("generated_tokens", 0) * world_scale(ctx) / mx, 1),
                "typeCorrections": int(st.get("type_corrections", 0)), "splitClasses": int(st.get("split_classes", 0)),
                "methodsDropped": int(st.get("methods_dropped", 0)),
                "classesAnalyzed": int(tot[1]), "elapsedS": round(mx, 3), "enrichFailed": r.stats.get("enrichFailed"),
                "phase2Ms": round(r.stats.get("analyze.phase2", 0.0), 1),
                "decodeStepMs": round(1e3 * st.get("decode_s", 0) / steps, 3),
                "hostMsPerStep": round(1e3 * st.get("host_s", 0) / steps, 3),
                "launchMsPerStep": round(1e3 * st.get("launch_s", 0) / steps, 3),
                "waitMsPerStep": round(1e3 * st.get("wait_s", 0) / steps, 3),
                "rowsPerStep": round(st.get("decode_rows", 0) / steps, 1),
                "prefillMsPerClass": round(1e3 * st.get("prefill_s", 0) / max(1, st.get("prefills", 0)), 3),
                "prefillBatches": int(st.get("prefill_batches", 0)), "workerInitS": round(init_s, 1),
                "config": {"model": f"{pool.model['preset']} (random init)", "kv_dtype": args.enrich_local_kv,
                           "prefill_dtype": args.enrich_local_prefill,
                           "batch": args.enrich_local_batch, "workers_per_rank": len(pool.workers),
                           "path": "analyze_project -> streamed Phase 2 -> GPU worker process"}}
    finally:
        app.db.close()


def _enrich_pool(pool, args, work) -> dict:
    """extra.enrichLocalPool: the production layout -- ONE project dealt by
    ONE GpuWorkerPool over every GPU of the job (dmcp/enrich/workers.py:
    classes dealt evenly, one worker process per GPU), run by rank 0 alone
    after the per-rank runs.  With --gpus 1, 2, 4, 8 the driver's runs give
    this fixed-size project's strong-scaling curve."""
    from dmcp.app import App
    from dmcp.config import Config
    from dmcp.enrich.workers import ProcessLLMBackend
    from dmcp.utils import synth
    t_init = time.perf_counter()
    pool.init()
    init_s = time.perf_counter() - t_init
    be = ProcessLLMBackend(pool)
    cfg = Config(db_path=os.path.join(work, "pool.db"), git_clone_base_path=os.path.join(work, "pclones"),
                 require_enrichment_for_analyze=True, recover_stuck_on_start=False)
    app = App(cfg, backend=be)
    try:
        warm = os.path.join(work, "poolwarm")
        synth.java_spring_repo(warm, n_classes=8 * len(pool.workers), base_package="co.acme.pwarm", seed=401)
        app.indexer.analyze_project(warm)  # every worker's first batch (allocator, first replays)
        repo = os.path.join(work, "poolrepo")
        synth.java_spring_repo(repo, n_classes=args.pool_classes, base_package="co.acme.pool", seed=402)
        for w in pool.workers:
            w.stats = {}
        pool.per_worker_items = {}
        t0 = time.perf_counter()
        r = app.indexer.analyze_project(repo)
        el = time.perf_counter() - t0
        st = be.stats()
        per = dict(getattr(pool, "per_worker_items", {}) or {})
        return {"classesPerSec": round(r.classes_analyzed / el, 2), "classes": r.classes_analyzed,
                "enriched": int(r.stats.get("enriched", 0)), "enrichFailed": r.stats.get("enrichFailed"),
                "elapsedS": round(el, 3), "phase2S": round(r.stats.get("analyze.phase2", 0.0) / 1e3, 3),
                "workers": len(pool.workers), "classesPerWorker": {str(k): v for k, v in sorted(per.items())},
                "generatedTokensPerSec": round(st.get("generated_tokens", 0) / el, 1),
                "decodeSteps": int(st.get("decode_steps", 0)), "workerInitS": round(init_s, 1),
                "config": {"model": f"{pool.model['preset']} (random init)", "kv_dtype": args.enrich_local_kv,
                           "batch": args.enrich_local_batch,
                           "path": "analyze_project -> streamed Phase 2 -> ONE GpuWorkerPool, one worker per GPU"}}
    finally:
        app.db.close()


def _lang_index(kind: str, args, work: str, threads: int) -> dict:
    """extra.tsIndex / extra.goIndex: the production analyze_project of a
    generated TypeScript (NestJS, reference NodeJsGraalParser.java:102-189)
    or Go (gin, reference GoSourceParser.java:339-372) repository of
    ``--lang-files`` source files, enrichment off, timed over
    ``--lang-steps`` analyses after one warm-up -- BASELINE configs 4-5 at
    scale."""
    from dmcp.app import App
    from dmcp.config import Config
    from dmcp.utils import synth
    root = os.path.join(work, f"{kind}repo")
    if kind == "ts":
        synth.nestjs_repo(root, n_modules=max(1, args.lang_files // 4))
        ext = (".ts",)
    else:
        synth.go_service_repo(root, n_packages=max(1, args.lang_files // 4))
        ext = (".go",)
    files = sum(1 for r, _, fs in os.walk(root) if "/.git" not in r for f in fs if f.endswith(ext))
    cfg = Config(db_path=os.path.join(work, f"{kind}.db"), git_clone_base_path=os.path.join(work, f"{kind}clones"),
                 parser_threads=threads, enrich_backend="null", require_enrichment_for_analyze=False,
                 recover_stuck_on_start=False)
    app = App(cfg)
    try:
        app.indexer.analyze_project(root)  # warm-up
        t0 = time.perf_counter()
        acc = {}
        for _ in range(args.lang_steps):
            r = app.indexer.analyze_project(root)
            for k, v in r.stats.items():
                if k.startswith("analyze."):
                    acc[k] = acc.get(k, 0.0) + v
        el = time.perf_counter() - t0
        return {"sourceFiles": files, "classesPerRepo": r.classes_analyzed,
                "msPerAnalysis": round(1e3 * el / args.lang_steps, 2),
                "filesPerSec": round(files * args.lang_steps / el, 1),
                "classesPerSec": round(r.classes_analyzed * args.lang_steps / el, 1),
                "phaseMs": {k: round(v / args.lang_steps, 2) for k, v in acc.items()},
                "framework": "nestjs" if kind == "ts" else "gin", "steps": args.lang_steps}
    finally:
        app.close()


def _remote_path(args, work, repo, threads):
    """extra.remotePath: the production path of a REMOTE repository, timed --
    a private bare clone (``git clone --bare --depth 1``, never the local
    objects in place) + the source scan in an isolated child process with its
    time limit (dmcp/parsers/isolated.py) + Phase 1 + graph publish.  The
    repository is a local one (no network here), so the clone is a local
    transport: the cost of the clone machinery and the child scan, not of a
    network."""
    from dmcp.app import App
    from dmcp.config import Config
    cfg = Config(db_path=os.path.join(work, "remote.db"), git_clone_base_path=os.path.join(work, "rclones"),
                 parser_threads=threads, enrich_backend="null", require_enrichment_for_analyze=False,
                 recover_stuck_on_start=False, scan_isolation="process")
    app = App(cfg)
    app.git.read_local_in_place = False
    try:
        app.indexer.analyze_project(repo)  # warm-up
        t0 = time.perf_counter()
        acc = {}
        for _ in range(args.remote_steps):
            r = app.indexer.analyze_project(repo)
            for k, v in r.stats.items():
                if k.startswith("analyze."):
                    acc[k] = acc.get(k, 0.0) + v
        el = time.perf_counter() - t0
        return {"msPerAnalysis": round(1e3 * el / args.remote_steps, 2),
                "classesPerSec": round(r.classes_analyzed * args.remote_steps / el, 1),
                "phaseMs": {k: round(v / args.remote_steps, 2) for k, v in acc.items()},
                "path": "bare clone (local transport) + isolated child scan + Phase 1"}
    finally:
        app.close()


def main(argv=None) -> int:
    args = parse_args(argv)
    pools = _spawn_enrich_pools(args) if args.enrich == "none" else {}  # before anything touches HIP
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
        for kind in (("ts", "go") if rank == 0 and args.lang_files > 0 else ()):
            key = "tsIndex" if kind == "ts" else "goIndex"
            try:
                extra[key] = _lang_index(kind, args, work, threads)
            except Exception as e:
                logging.getLogger("bench").exception("%s failed", key)
                extra[key] = {"error": repr(e)[:300]}
        if rank == 0 and args.remote_steps > 0:
            try:
                extra["remotePath"] = _remote_path(args, work, repo, threads)
            except Exception as e:
                logging.getLogger("bench").exception("remotePath failed")
                extra["remotePath"] = {"error": repr(e)[:300]}
        # agreed by every rank: a rank without a worker skips the collective path for all
        names = [p.strip() for p in args.enrich_local_presets.split(",") if p.strip()]
        have = sum(1 for n in names if n in pools)  # the per-rank preset workers (not rank 0's pool)
        if args.enrich == "none" and args.enrich_local_classes > 0 and \
                ctx.sum(1.0 if have == len(names) else 0.0)[0] == world:
            for name in names:
                key = EXTRA_KEYS.get(name, "enrichLocal_" + name)
                try:
                    extra[key] = _enrich_local(pools[name], args, ctx, work, rank)
                except Exception as e:
                    logging.getLogger("bench").exception("%s failed", key)
                    extra[key] = {"error": repr(e)[:300]}
                finally:
                    pools.pop(name).close()  # its KV slab goes before the next preset's
        if POOL_KEY in pools:  # rank 0 only; no collective inside
            try:
                extra["enrichLocalPool"] = _enrich_pool(pools[POOL_KEY], args, work)
            except Exception as e:
                logging.getLogger("bench").exception("enrichLocalPool failed")
                extra["enrichLocalPool"] = {"error": repr(e)[:300]}
            finally:
                pools.pop(POOL_KEY).close()
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
        for p in pools.values():
            p.close()
        if args.workdir is None:
            shutil.rmtree(work, ignore_errors=True)
        ctx.shutdown()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
