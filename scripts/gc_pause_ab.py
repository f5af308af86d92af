"""Interleaved A/B (one process) of the indexer's GC pause
(dmcp/utils/runtime.py GcPause): the 2,001-class bench repository analysed
with the pause on and off in alternating rounds, on the local fast path and
on the remote path (bare clone + isolated child scan).  Prints one JSON line
per path: median / min ms per analysis and the median analyze.* phases.

  python scripts/gc_pause_ab.py [--rounds 6] [--per 5]
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
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--per", type=int, default=5)
    ap.add_argument("--classes", type=int, default=2000)
    args = ap.parse_args()
    import torch  # noqa: F401  (bench.py's process has it imported: ~10^6 long-lived objects)
    from dmcp.app import App
    from dmcp.config import Config
    from dmcp.utils import runtime, synth
    work = tempfile.mkdtemp(prefix="dmcp-gcab-")
    repo = os.path.join(work, "shop0")
    synth.java_spring_repo(repo, n_classes=args.classes, base_package="co.acme.shop0", seed=1)
    orig = runtime.GcPause.start
    med = lambda v: sorted(v)[len(v) // 2]
    try:
        for path in ("local", "remote"):
            cfg = Config(db_path=os.path.join(work, f"{path}.db"), git_clone_base_path=os.path.join(work, f"c-{path}"),
                         parser_threads=8, enrich_backend="null", require_enrichment_for_analyze=False,
                         recover_stuck_on_start=False, scan_isolation="process" if path == "remote" else "auto")
            app = App(cfg)
            if path == "remote":
                app.git.read_local_in_place = False
            for _ in range(3):
                app.indexer.analyze_project(repo)
            ms = {"on": [], "off": []}
            ph = {"on": {}, "off": {}}
            for _ in range(args.rounds):
                for mode in ("off", "on"):
                    runtime.GcPause.start = orig if mode == "on" else (lambda self: self)
                    for _ in range(args.per):
                        t0 = time.perf_counter()
                        r = app.indexer.analyze_project(repo)
                        ms[mode].append((time.perf_counter() - t0) * 1e3)
                        for k, v in r.stats.items():
                            if k.startswith("analyze."):
                                ph[mode].setdefault(k, []).append(v)
            runtime.GcPause.start = orig
            app.close()
            print(json.dumps({"path": path, "classes": r.classes_analyzed,
                              **{mode: {"median_ms": round(med(v), 2), "min_ms": round(min(v), 2),
                                        "phases": {k: round(med(x), 2) for k, x in ph[mode].items()}}
                                 for mode, v in ms.items()}}), flush=True)
    finally:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
