"""Command line: ``python -m dmcp <command>``.

Commands
  serve-mcp                      MCP stdio server (the reference's ``mcp`` profile)
  serve [--host H] [--port P]    REST API + Swagger + optional sync scheduler
  analyze URL [--branch B] [--no-fix-missed]
  analyze-batch FILE [--workers N]  bulk index 'url [branch]' lines; exit code = failures
  rebuild PROJECT_ID             re-parse without enrichment
  delete PROJECT_ID              remove a project and its classes / graph
  resume PROJECT_ID              re-enrich classes with no description
  sync [--project NAME]          incremental git-diff sync (all eligible by default)
  query "project:target..."      graph DSL
  tool NAME [JSON_ARGS]          call any MCP tool and print its JSON
  list                           list_projects
  scan ROOT [--lang L]           native front-end output (JSON)
  stats                          metrics snapshot of this process
"""
from __future__ import annotations

import argparse
import json
import sys
from typing import List, Optional


def _app(args):
    from .app import App, configure_logging
    from .config import Config
    cfg = Config.from_env()
    if getattr(args, "db", None):
        cfg = cfg.merged({"db_path": args.db})
    configure_logging(cfg.log_level)
    return App(cfg)


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(prog="dmcp", description="Domain-aware code-graph MCP server")
    ap.add_argument("--db", help="SQLite database path (default: $DMCP_DB_PATH or ~/.dmcp/dmcp.db)")
    sub = ap.add_subparsers(dest="cmd", required=True)
    sub.add_parser("serve-mcp")
    s = sub.add_parser("serve")
    s.add_argument("--host")
    s.add_argument("--port", type=int)
    a = sub.add_parser("analyze")
    a.add_argument("url")
    a.add_argument("--branch")
    a.add_argument("--no-fix-missed", action="store_true")
    ab = sub.add_parser("analyze-batch")
    ab.add_argument("file", help="repos.txt: 'url [branch]' per line")
    ab.add_argument("--workers", type=int, default=1)
    ab.add_argument("--no-fix-missed", action="store_true")
    r = sub.add_parser("rebuild")
    r.add_argument("project_id")
    dl = sub.add_parser("delete")
    dl.add_argument("project_id")
    rs = sub.add_parser("resume")
    rs.add_argument("project_id")
    sy = sub.add_parser("sync")
    sy.add_argument("--project")
    q = sub.add_parser("query")
    q.add_argument("query")
    t = sub.add_parser("tool")
    t.add_argument("name")
    t.add_argument("arguments", nargs="?", default="{}")
    sub.add_parser("list")
    sc = sub.add_parser("scan")
    sc.add_argument("root")
    sc.add_argument("--lang", default="auto")
    sc.add_argument("--threads", type=int, default=0)
    sub.add_parser("stats")
    args = ap.parse_args(argv)

    if args.cmd == "scan":
        from .parsers.base import native
        sys.stdout.write(native().scan_project(args.root, args.lang, args.threads, "").decode() + "\n")
        return 0
    if args.cmd == "serve-mcp":
        from .api.mcp_stdio import McpServer
        app = _app(args)
        try:
            McpServer(app).serve()
        finally:
            app.close()
        return 0
    if args.cmd == "serve":
        from .api.rest import serve
        app = _app(args)
        serve(app, args.host, args.port)
        return 0
    app = _app(args)
    try:
        out = None
        if args.cmd == "analyze":
            out = app.indexer.analyze_project(args.url, args.branch, not args.no_fix_missed).to_dict()
        elif args.cmd == "analyze-batch":
            from dataclasses import asdict
            from .parallel.bulk import bulk_analyze, parse_repo_list
            with open(args.file, encoding="utf-8") as f:
                items = parse_repo_list(f.read())
            res = bulk_analyze(app.config, items, args.workers, not args.no_fix_missed, app=app)
            failed = sum(1 for x in res if not x.success)
            print(json.dumps({"total": len(res), "success": len(res) - failed, "failed": failed,
                              "results": [asdict(x) for x in res]}, indent=2))
            return failed  # exit code = number of failures (analyze-repos.sh parity)
        elif args.cmd == "delete":
            ok = app.projects.delete_project(args.project_id)
            out = {"success": ok, "projectId": args.project_id,
                   "message": "Project deleted" if ok else "Project not found"}
            if not ok:
                print(json.dumps(out))
                return 1
        elif args.cmd == "rebuild":
            out = app.indexer.rebuild_graph(args.project_id)
        elif args.cmd == "resume":
            out = app.indexer.resume_enrichment(args.project_id)
        elif args.cmd == "sync":
            if args.project:
                p = app.repos.projects.find_by_name(args.project)
                if p is None:
                    print(json.dumps({"success": False, "errorMessage": f"Project not found: {args.project}"}))
                    return 1
                out = app.indexer.sync_project(p).to_dict()
            else:
                r = app.indexer.sync_all_projects()
                out = {"success": r.success, "totalProjects": r.total_projects, "successCount": r.success_count,
                       "failureCount": r.failure_count, "results": [x.to_dict() for x in r.results]}
        elif args.cmd == "query":
            out = app.graph_query.query(args.query).to_dict()
        elif args.cmd == "tool":
            from .api.tools import ToolRegistry
            res = ToolRegistry(app).call(args.name, json.loads(args.arguments))
            text = res["content"][0]["text"]
            print(text if res["isError"] else json.dumps(json.loads(text), indent=2))
            return 1 if res["isError"] else 0
        elif args.cmd == "list":
            out = app.context.list_projects()
        elif args.cmd == "stats":
            from .utils.tracing import METRICS
            out = METRICS.snapshot()
        print(json.dumps(out, indent=2, default=str))
        return 0
    except Exception as e:
        from .utils.errors import DomainError
        if isinstance(e, DomainError):
            print(json.dumps({"error": e.message, "errorCode": e.error_code}))
            return 2
        raise
    finally:
        app.close()


if __name__ == "__main__":
    raise SystemExit(main())
