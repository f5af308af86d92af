#!/usr/bin/env python3
"""The five BASELINE.json configurations, measured end to end on this host.

1. Index a 10-file toy Java Spring repo, then ``list_projects`` over MCP stdio
   (a real ``python -m dmcp serve-mcp`` child process, JSON-RPC over pipes).
2. ``search_project`` + ``get_class_context`` on a ~200-class Java monorepo.
3. ``get_stack_trace_context`` for a 20-frame Java stack trace.
4. Index a NestJS TypeScript service, then a ``graph_query`` DSL path query.
5. Index a Go (gin) service alongside 2 Java services; cross-project
   ``get_class_dependencies``.

Plus indexing throughput per language (classes/s and files/s, enrichment
off).  Prints one JSON object per line; ``--out`` also writes them to a file.
Synthetic repositories (``dmcp.utils.synth``), no network, no LLM.

    python scripts/bench_configs.py [--iters 200] [--out profiles/configs.jsonl]
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from dmcp.app import App  # noqa: E402
from dmcp.config import Config  # noqa: E402
from dmcp.utils import synth  # noqa: E402


def pct(xs, p):
    xs = sorted(xs)
    return round(xs[min(len(xs) - 1, max(0, int(round(p / 100 * len(xs))) - 1))], 3)


def timed(fn, iters):
    lat = []
    for _ in range(iters):
        t0 = time.perf_counter()
        fn()
        lat.append((time.perf_counter() - t0) * 1e3)
    return {"p50_ms": pct(lat, 50), "p99_ms": pct(lat, 99), "n": iters}


def index_rate(app, repo, files, reps=3):
    best = None
    for _ in range(reps):
        r = app.indexer.analyze_project(repo)
        ms = r.stats["analyze.total"]
        if best is None or ms < best[0]:
            best = (ms, r)
    ms, r = best
    return r, {"classes": r.classes_analyzed, "files": files, "analyze_ms": round(ms, 2),
               "classes_per_s": round(r.classes_analyzed / ms * 1e3, 1), "files_per_s": round(files / ms * 1e3, 1),
               "endpoints": r.endpoints_found}


def count_files(root, exts):
    n = 0
    for d, dirs, fs in os.walk(root):
        dirs[:] = [x for x in dirs if x not in (".git", "node_modules")]
        n += sum(1 for f in fs if f.endswith(exts))
    return n


class McpClient:
    """JSON-RPC 2.0 over a child ``serve-mcp`` process's stdio."""

    def __init__(self, env):
        self.p = subprocess.Popen([sys.executable, "-m", "dmcp", "serve-mcp"], cwd=ROOT, env=env,
                                  stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL,
                                  text=True, bufsize=1)
        self.id = 0

    def call(self, method, params=None):
        self.id += 1
        self.p.stdin.write(json.dumps({"jsonrpc": "2.0", "id": self.id, "method": method,
                                       "params": params or {}}) + "\n")
        self.p.stdin.flush()
        resp = json.loads(self.p.stdout.readline())
        if "error" in resp:
            raise RuntimeError(resp["error"])
        return resp["result"]

    def close(self):
        self.p.stdin.close()
        self.p.wait(timeout=30)


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    threads = a.threads or max(1, min(16, os.cpu_count() or 8))
    work = tempfile.mkdtemp(prefix="dmcp-configs-")
    lines = []

    def emit(rec):
        lines.append(rec)
        print(json.dumps(rec), flush=True)

    def make_app(name):
        return App(Config(db_path=os.path.join(work, f"{name}.db"), git_clone_base_path=os.path.join(work, "c"),
                          parser_threads=threads, enrich_backend="null", require_enrichment_for_analyze=False,
                          recover_stuck_on_start=False))
    try:
        # ---- config 1: toy repo + list_projects over MCP stdio
        toy = os.path.join(work, "toy")
        synth.java_spring_repo(toy, 10, base_package="co.acme.toy")
        app = make_app("c1")
        t0 = time.perf_counter()
        r = app.indexer.analyze_project(toy)
        index_ms = (time.perf_counter() - t0) * 1e3
        app.close()
        env = dict(os.environ, DATABASE_URL=f"sqlite:///{os.path.join(work, 'c1.db')}", READ_ONLY="true",
                   ANTHROPIC_API_KEY="")
        t0 = time.perf_counter()
        mcp = McpClient(env)
        mcp.call("initialize", {"protocolVersion": "2024-11-05", "capabilities": {},
                                "clientInfo": {"name": "bench", "version": "1"}})
        start_ms = (time.perf_counter() - t0) * 1e3
        res = mcp.call("tools/call", {"name": "list_projects", "arguments": {}})
        listed = json.loads(res["content"][0]["text"])
        lat = timed(lambda: mcp.call("tools/call", {"name": "list_projects", "arguments": {}}), a.iters)
        mcp.close()
        emit({"config": 1, "name": "toy Java repo + list_projects over MCP stdio", "classes": r.classes_analyzed,
              "index_ms": round(index_ms, 2), "mcp_start_ms": round(start_ms, 1),
              "projects_listed": len(listed.get("projects", listed) if isinstance(listed, dict) else listed),
              "list_projects": lat})

        # ---- configs 2 + 3: ~200-class monorepo
        mono = os.path.join(work, "shop")
        fqcns = synth.java_spring_repo(mono, 200)
        app = make_app("c2")
        r, rate = index_rate(app, mono, count_files(mono, (".java",)))
        fq = fqcns[len(fqcns) // 2]
        assert app.context.get_class_context(fq)["found"] and app.context.search_project("shop", "Order")["matches"]
        emit({"config": 2, "name": "search_project + get_class_context, 200-class monorepo", "index": rate,
              "search_project": timed(lambda: app.context.search_project("shop", "Order"), a.iters),
              "get_class_context": timed(lambda: app.context.get_class_context(fq), a.iters)})
        trace = synth.stack_trace_for(fqcns, 20)
        emit({"config": 3, "name": "get_stack_trace_context, 20 frames",
              "get_stack_trace_context": timed(lambda: app.context.get_stack_trace_context(trace), a.iters)})
        app.close()

        # ---- config 4: NestJS + graph_query path
        nest = os.path.join(work, "nest")
        synth.nestjs_repo(nest, 40)
        app = make_app("c4")
        r, rate = index_rate(app, nest, count_files(nest, (".ts", ".tsx", ".js", ".jsx")))
        g = app.cache.get_graph(r.project_id)
        src = next(i for i in g.entry_points() if g.dependencies(i))
        # path: entry point -> its dependencies, with their methods and logic
        q = f"nest:{src}:dependencies:+methods:+logic"
        assert app.graph_query.query(q).count > 0
        emit({"config": 4, "name": "NestJS index + graph_query path query", "index": rate, "query": q,
              "graph_query": timed(lambda: app.graph_query.query(q), a.iters)})
        app.close()

        # ---- config 5: Go (gin) + 2 Java services, cross-project dependencies
        app = make_app("c5")
        gosvc = os.path.join(work, "gosvc")
        synth.go_gin_repo(gosvc, 24)
        _, go_rate = index_rate(app, gosvc, count_files(gosvc, (".go",)))
        java_rates = []
        java_fq = []
        for i in range(2):
            p = os.path.join(work, f"svc{i}")
            java_fq.append(synth.java_spring_repo(p, 150, base_package=f"co.acme.svc{i}", seed=i + 3))
            _, jr = index_rate(app, p, count_files(p, (".java",)), reps=1)
            java_rates.append(jr)
        target = next(f for f in java_fq[1] if app.context.get_class_dependencies(f)["dependencies"])
        emit({"config": 5, "name": "Go (gin) + 2 Java services, cross-project get_class_dependencies",
              "index_go": go_rate, "index_java": java_rates,
              "get_class_dependencies": timed(lambda: app.context.get_class_dependencies(target), a.iters)})
        app.close()
    finally:
        shutil.rmtree(work, ignore_errors=True)
    if a.out:
        with open(a.out, "w") as f:
            for rec in lines:
                f.write(json.dumps(rec) + "\n")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
