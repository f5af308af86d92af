"""Bulk repository indexing.

Parity: ``scripts/analyze-repos.sh:18-80`` reads ``repos.txt`` (``url
[branch]`` per line, ``#`` comments) and POSTs ``/api/projects/analyze`` for
each repository *sequentially* with ``fixMissed: true``; the exit code is the
number of failures.  Here the same list can be indexed in-process, optionally
across ``workers`` processes: each worker opens its own connection to the
shared SQLite file (WAL, ``BEGIN IMMEDIATE`` writers), so clone + native parse
+ graph build of different repositories run in parallel and only the Phase 1
swap transactions serialise.
"""
from __future__ import annotations

import logging
import os
from concurrent.futures import ProcessPoolExecutor, as_completed
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


def bulk_analyze(config, items: Sequence[BulkItem], workers: int = 1, fix_missed: bool = True,
                 app=None) -> List[BulkResult]:
    """Analyzes every repository; returns results in input order.

    ``workers == 1`` runs in this process (reusing ``app`` when given);
    ``workers > 1`` uses a process pool, each process with its own App."""
    results: List[Optional[BulkResult]] = [None] * len(items)
    if workers <= 1 or len(items) <= 1:
        from ..app import App
        own = app is None
        app = app or App(config)
        try:
            for i, it in enumerate(items):
                try:
                    r = app.indexer.analyze_project(it.url, it.branch, fix_missed)
                    results[i] = BulkResult(it.url, r.success, r.project_id, r.classes_analyzed,
                                            r.endpoints_found, r.message)
                except Exception as e:
                    results[i] = BulkResult(it.url, False, None, 0, 0, getattr(e, "message", str(e)))
                LOG.info("[%d/%d] %s -> %s", i + 1, len(items), it.url, "ok" if results[i].success else "FAILED")
        finally:
            if own:
                app.close()
        return results  # type: ignore[return-value]
    values = {k: getattr(config, k) for k in config.__dataclass_fields__}
    values["recover_stuck_on_start"] = False  # siblings may be mid-analysis
    from ..store.db import Database
    Database(config.db_path).close()  # create + migrate once, before the workers race for it
    with ProcessPoolExecutor(max_workers=min(workers, len(items), os.cpu_count() or 1)) as ex:
        futs = {ex.submit(_analyze_one, values, (it.url, it.branch), fix_missed): i for i, it in enumerate(items)}
        for f in as_completed(futs):
            results[futs[f]] = BulkResult(**f.result())
    return results  # type: ignore[return-value]
