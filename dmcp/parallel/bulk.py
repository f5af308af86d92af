"""Bulk repository indexing.

Parity: ``scripts/analyze-repos.sh:18-80`` reads ``repos.txt`` (``url
[branch]`` per line, ``#`` comments) and POSTs ``/api/projects/analyze`` for
each repository *sequentially* with ``fixMissed: true``; the exit code is the
number of failures.  Here the same list can be indexed in-process, ``workers``
repositories at a time:

* with the local MI355X enrichment backend the repositories run on threads of
  ONE application, so they share its one GPU worker pool (one process per
  GPU, each with its model and KV slab): the pool splits the GPUs over the
  projects being enriched at the moment -- a pool per repository would load
  the model and allocate the KV slab again for every one of them;
* otherwise on a process pool: each process opens its own connection to the
  shared store (SQLite WAL with ``BEGIN IMMEDIATE`` writers, or PostgreSQL),
  so clone + native parse + graph build of different repositories run in
  parallel and only the Phase 1 swap transactions serialise.
"""
from __future__ import annotations

import logging
import os
from concurrent.futures import ProcessPoolExecutor, ThreadPoolExecutor, as_completed
from dataclasses import asdict, dataclass
from typing import Dict, List, Optional, Sequence, Tuple

LOG = logging.getLogger(__name__)


@dataclass
class BulkItem:
    url: str
    branch: Optional[str] = None


@dataclass
class BulkResult:
    url: str
    success: bool
    project_id: Optional[str]
    classes: int
    endpoints: int
    message: str


def parse_repo_list(text: str) -> List[BulkItem]:
    """``url [branch]`` per line; blank lines and ``#`` comments skipped."""
    items = []
    for line in text.splitlines():
        line = line.strip()
        if not line or line.startswith("#"):
            continue
        parts = line.split()
        items.append(BulkItem(parts[0], parts[1] if len(parts) > 1 else None))
    return items


def _analyze_one(config_values: Dict, item: Tuple[str, Optional[str]], fix_missed: bool) -> Dict:
    from ..app import App
    from ..config import Config
    url, branch = item
    app = App(Config().merged(config_values), load_graphs=False)
    try:
        r = app.indexer.analyze_project(url, branch, fix_missed)
        return asdict(BulkResult(url, r.success, r.project_id, r.classes_analyzed, r.endpoints_found, r.message))
    except Exception as e:
        msg = getattr(e, "message", str(e))
        return asdict(BulkResult(url, False, None, 0, 0, msg))
    finally:
        app.close()


def _run_one(app, it: BulkItem, fix_missed: bool) -> BulkResult:
    try:
        r = app.indexer.analyze_project(it.url, it.branch, fix_missed)
        return BulkResult(it.url, r.success, r.project_id, r.classes_analyzed, r.endpoints_found, r.message)
    except Exception as e:
        return BulkResult(it.url, False, None, 0, 0, getattr(e, "message", str(e)))


def shares_one_app(config, workers: int, n_items: int) -> bool:
    """True when the repositories run on threads of one application: a
    single worker, or the local GPU backend (one pool for all of them)."""
    return workers <= 1 or n_items <= 1 or config.resolved_enrich_backend() == "local"


def bulk_analyze(config, items: Sequence[BulkItem], workers: int = 1, fix_missed: bool = True,
                 app=None) -> List[BulkResult]:
    """Analyzes every repository; returns results in input order.

    One application (``app``, or one built here) serves every repository
    when :func:`shares_one_app` -- ``workers`` threads over it; else a pool
    of ``workers`` processes, each with its own App."""
    results: List[Optional[BulkResult]] = [None] * len(items)
    if shares_one_app(config, workers, len(items)):
        from ..app import App
        own = app is None
        app = app or App(config)
        try:
            if workers <= 1 or len(items) <= 1:
                for i, it in enumerate(items):
                    results[i] = _run_one(app, it, fix_missed)
                    LOG.info("[%d/%d] %s -> %s", i + 1, len(items), it.url,
                             "ok" if results[i].success else "FAILED")
            else:
                with ThreadPoolExecutor(max_workers=min(workers, len(items)), thread_name_prefix="bulk") as ex:
                    futs = {ex.submit(_run_one, app, it, fix_missed): i for i, it in enumerate(items)}
                    for n, f in enumerate(as_completed(futs), 1):
                        i = futs[f]
                        results[i] = f.result()
                        LOG.info("[%d/%d] %s -> %s", n, len(items), items[i].url,
                                 "ok" if results[i].success else "FAILED")
        finally:
            if own:
                app.close()
        return results  # type: ignore[return-value]
    values = {k: getattr(config, k) for k in config.__dataclass_fields__}
    values["recover_stuck_on_start"] = False  # siblings may be mid-analysis
    if not config.database_url:  # SQLite: create + migrate once, before the workers race for it
        from ..store.db import Database
        Database(config.db_path).close()
    with ProcessPoolExecutor(max_workers=min(workers, len(items), os.cpu_count() or 1)) as ex:
        futs = {ex.submit(_analyze_one, values, (it.url, it.branch), fix_missed): i for i, it in enumerate(items)}
        for f in as_completed(futs):
            results[futs[f]] = BulkResult(**f.result())
    return results  # type: ignore[return-value]
