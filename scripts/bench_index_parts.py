#!/usr/bin/env python3
"""Sub-steps of one analysis' snapshot + parse on the bench repository
(2,000-class synthetic Spring monorepo), medians over repeats, with a thread
sweep of the native stages.  One JSON line per (stage, threads).

    python scripts/bench_index_parts.py [--classes 2000] [--reps 9]
"""
import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dmcp import _srcscan as N  # noqa: E402
from dmcp.index import source as S  # noqa: E402
from dmcp.index.git import GitClient  # noqa: E402
from dmcp.models.domain import StaticMethodInfo  # noqa: E402
from dmcp.utils import synth  # noqa: E402


def med(fn, reps):
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t) * 1e3)
    return round(sorted(ts)[len(ts) // 2], 3)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--classes", type=int, default=2000)
    ap.add_argument("--reps", type=int, default=9)
    a = ap.parse_args()
    work = tempfile.mkdtemp(prefix="dmcp-parts-")
    repo = os.path.join(work, "shop")
    synth.java_spring_repo(repo, a.classes)
    g = GitClient(os.path.join(work, "c"))
    c = g.resolve_commit(repo, None)
    ents = [e for e in S.list_tree(g, repo, c) if S.wanted(e[0])]
    dirs = S._object_dirs(repo)
    shas = [e[1] for e in ents]
    blobs = N.read_loose_blobs(dirs, shas, 16, 0)[0]
    items = list(zip([e[0] for e in ents], blobs))
    out = {"cpus": os.cpu_count(), "files": len(items), "bytes": sum(len(b) for b in blobs)}
    print(json.dumps(out), flush=True)
    rows = [("rev-parse", 0, lambda: g.resolve_commit(repo, None)),
            ("ls-tree", 0, lambda: S.list_tree(g, repo, c)),
            ("mostly_loose", 0, lambda: S.mostly_loose(repo))]
    if hasattr(N, "list_tree_loose"):
        rows.append(("native_tree", 0, lambda: N.list_tree_loose(dirs, c)))
    if hasattr(N, "resolve_ref"):
        rows.append(("native_ref", 0, lambda: N.resolve_ref(S.git_dir_of(repo), ["HEAD"])))
    for th in (1, 4, 8, 16, 32):
        rows.append(("read_loose", th, lambda th=th: N.read_loose_blobs(dirs, shas, th, 0)))
        rows.append(("scan_objects", th, lambda th=th: N.scan_sources_objects(items, "java", th, "",
                                                                                  StaticMethodInfo)))
        rows.append(("scan_json", th, lambda th=th: N.scan_sources(items, "java", th, "")))
    for name, th, fn in rows:
        fn()
        rec = {"stage": name, "threads": th, "ms": med(fn, a.reps)}
        if name == "scan_objects":
            st = fn()["stats"]
            rec["phase_ms"] = {k: v / 1e3 for k, v in st.get("phaseUs", {}).items()}
            rec["native_ms"] = st["elapsedUs"] / 1e3
        print(json.dumps(rec), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
