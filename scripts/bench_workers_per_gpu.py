"""Engines per GPU A/B: one project dealt by a GpuWorkerPool with 1 or 2
worker processes on the SAME GPU (each with half the KV slots), alternating.
Small projects are latency-bound (a ~100-row decode step leaves most of the
chip idle between its short kernels); this measures whether two independent
engine streams on one GPU overlap those gaps.  One JSON line per run.

  python scripts/bench_workers_per_gpu.py [--preset llama3.2-1b-code] [--classes 34 257] [--rounds 2]
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="llama3.2-1b-code")
    ap.add_argument("--classes", type=int, nargs="+", default=[34, 257])
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--batch", type=int, default=768, help="KV slots per GPU (split over its workers)")
    ap.add_argument("--workers", type=int, nargs="+", default=[1, 2])
    args = ap.parse_args()
    from dmcp.app import App
    from dmcp.config import Config
    from dmcp.enrich.workers import GpuWorkerPool, ProcessLLMBackend
    from dmcp.utils import synth
    work = tempfile.mkdtemp(prefix="dmcp-wpg-")
    repos = {}
    for n in args.classes:
        repos[n] = os.path.join(work, f"repo{n}")
        synth.java_spring_repo(repos[n], n_classes=n, base_package=f"co.acme.w{n}", seed=500 + n)
    warm = os.path.join(work, "warm")
    synth.java_spring_repo(warm, n_classes=16, base_package="co.acme.wwarm", seed=499)
    try:
        for rnd in range(args.rounds):
            for nw in args.workers:
                mb = args.batch // nw
                model = {"preset": args.preset, "kv_dtype": "fp8", "prefill_dtype": "auto", "max_batch": mb,
                         "max_rows": max(mb, min(1024, max(256, mb * 3 // 2))), "seed": 0}
                pool = GpuWorkerPool(["cuda:0"] * nw, model, engine={"max_new_tokens": 4096}, init=False,
                                     start_timeout_s=600)
                try:
                    t0 = time.perf_counter()
                    pool.init()
                    init_s = time.perf_counter() - t0
                    be = ProcessLLMBackend(pool)
                    cfg = Config(db_path=os.path.join(work, f"w{rnd}_{nw}.db"),
                                 git_clone_base_path=os.path.join(work, "clones"),
                                 require_enrichment_for_analyze=True, recover_stuck_on_start=False)
                    app = App(cfg, backend=be)
                    try:
                        app.indexer.analyze_project(warm)
                        for n, repo in repos.items():
                            for w in pool.workers:
                                w.stats = {}
                            t1 = time.perf_counter()
                            r = app.indexer.analyze_project(repo)
                            el = time.perf_counter() - t1
                            st = be.stats()
                            print(json.dumps({"bench": "workers_per_gpu", "preset": args.preset, "round": rnd,
                                              "workers": nw, "kv_slots_each": mb, "classes": r.classes_analyzed,
                                              "enriched": int(r.stats.get("enriched", 0)),
                                              "elapsedS": round(el, 3),
                                              "classesPerSec": round(r.classes_analyzed / el, 2),
                                              "generatedTokensPerSec": round(st.get("generated_tokens", 0) / el, 1),
                                              "decodeSteps": int(st.get("decode_steps", 0)),
                                              "initS": round(init_s, 1)}), flush=True)
                    finally:
                        app.db.close()
                finally:
                    pool.close()
    finally:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
