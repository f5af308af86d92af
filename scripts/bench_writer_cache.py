#!/usr/bin/env python3
"""How much of the row swap is the writer connection's cold page cache?

Replays one analysis' row swap (delete the project's 12.8k rows, insert them
again, commit) on the bench database: (a) on a fresh connection each time, as
the native bulk writer does, after another connection's small write (the
ANALYZING status update); (b) on one persistent connection with no foreign
write in between (its page cache stays valid).  Medians of --reps."""
import argparse
import json
import os
import sqlite3
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dmcp.app import App  # noqa: E402
from dmcp.config import Config  # noqa: E402
from dmcp.utils import synth  # noqa: E402

TABLES = ("source_classes", "source_methods", "method_parameters")


def swap(c, pid, rows, cols, repos) -> dict:
    t0 = time.perf_counter()
    c.execute("BEGIN IMMEDIATE")
    for r in (repos.params, repos.methods, repos.classes):
        c.execute(r.DELETE_BY_PROJECT_ID, (pid,))
    t1 = time.perf_counter()
    for t in TABLES:
        c.executemany(f"INSERT INTO {t} VALUES ({','.join('?' * cols[t])})", rows[t])
    t2 = time.perf_counter()
    c.execute("COMMIT")
    t3 = time.perf_counter()
    return {"delete": (t1 - t0) * 1e3, "insert": (t2 - t1) * 1e3, "commit": (t3 - t2) * 1e3}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=9)
    a = ap.parse_args()
    work = tempfile.mkdtemp(prefix="dmcp-wc-")
    repo = os.path.join(work, "shop")
    synth.java_spring_repo(repo, 2000)
    db = os.path.join(work, "db")
    app = App(Config(db_path=db, git_clone_base_path=os.path.join(work, "c"), enrich_backend="null",
                     require_enrichment_for_analyze=False, recover_stuck_on_start=False))
    r = app.indexer.analyze_project(repo)
    pid = r.project_id
    probe = sqlite3.connect(db)
    rows = {t: probe.execute(f"SELECT * FROM {t}").fetchall() for t in TABLES}
    cols = {t: len(v[0]) for t, v in rows.items()}
    probe.close()

    def conn():
        c = sqlite3.connect(db, isolation_level=None)
        for p in ("PRAGMA synchronous = NORMAL", "PRAGMA temp_store = MEMORY", "PRAGMA cache_size = -65536",
                  "PRAGMA foreign_keys = OFF", "PRAGMA wal_autocheckpoint = 0"):
            c.execute(p)
        return c
    other = conn()
    res = {"cold": [], "warm": []}
    for _ in range(a.reps):
        other.execute("UPDATE projects SET updated_at = updated_at WHERE id = ?", (pid,))  # a foreign commit
        c = conn()
        res["cold"].append(swap(c, pid, rows, cols, app.repos))
        c.close()
    c = conn()
    swap(c, pid, rows, cols, app.repos)
    for _ in range(a.reps):
        res["warm"].append(swap(c, pid, rows, cols, app.repos))
    for k, v in res.items():
        med = {f: round(sorted(x[f] for x in v)[len(v) // 2], 2) for f in ("delete", "insert", "commit")}
        print(json.dumps({"connection": k, "rows": sum(len(x) for x in rows.values()), **med}), flush=True)
    app.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
