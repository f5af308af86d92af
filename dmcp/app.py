"""Application container: wires config, storage, cache, parsers, enrichment and services.

Parity: the Spring context of ``DomainMcpServerApplication`` -- datasource +
migrations, repositories, ``CodeContextService``/``ProjectSyncService``
(sharing one enrichment client here instead of two independent semaphores,
SURVEY §3.1 step 2.5), ``GraphService.loadAll`` on start-up (``:55-76``) and the
optional ``ProjectSyncScheduler`` (``sync.enabled``).
"""
from __future__ import annotations

import logging
import sys
import threading
from typing import Optional

from .config import Config
from .enrich.backend import EnrichmentBackend, create_backend
from .graph.cache import GraphCache
from .index.git import GitClient
from .index.pipeline import Indexer
from .index.projects import ProjectService
from .models.domain import ProjectStatus
from .query.context import ContextService
from .query.dsl import GraphQueryService
from .store.db import Database
from .store.repositories import Repositories
from .utils.runtime import tune_gc

LOG = logging.getLogger(__name__)


class _StderrHandler(logging.StreamHandler):
    """Writes to whatever ``sys.stderr`` is at emit time (a redirected or
    replaced stderr -- test capture, daemonisation -- never sees writes to a
    stale, closed stream)."""

    def __init__(self) -> None:
        super().__init__(sys.stderr)

    @property  # type: ignore[override]
    def stream(self):
        return sys.stderr

    @stream.setter
    def stream(self, _value) -> None:
        pass


def configure_logging(level: str = "INFO", stream=None) -> None:
    """All logs go to stderr so stdout stays pure JSON-RPC in MCP mode
    (``logback-spring.xml:14-26``)."""
    root = logging.getLogger()
    if getattr(configure_logging, "_done", False):
        root.setLevel(level.upper())
        return
    h = logging.StreamHandler(stream) if stream is not None else _StderrHandler()
    h.setFormatter(logging.Formatter("%(asctime)s [%(threadName)s] %(levelname)-5s %(name)s - %(message)s",
                                     "%H:%M:%S"))
    root.handlers[:] = [h]
    root.setLevel(level.upper())
    configure_logging._done = True  # type: ignore[attr-defined]


def open_database(config: Config):
    """The store named by the configuration: PostgreSQL when ``database_url``
    is a PostgreSQL URL (the reference's own database), else SQLite at
    ``db_path``."""
    if config.database_url:
        from .store.pg import PgDatabase
        db = PgDatabase.from_url(config.database_url, config.database_username, config.database_password)
        LOG.info("Store: %s", db.describe())
        return db
    return Database(config.db_path, background_checkpoint=config.db_background_checkpoint)


class App:
    def __init__(self, config: Optional[Config] = None, *, backend: Optional[EnrichmentBackend] = None,
                 load_graphs: bool = True, db: Optional[Database] = None) -> None:
        self.config = config or Config.from_env()
        self.db = db or open_database(self.config)
        self.repos = Repositories(self.db)
        self.cache = GraphCache(self.repos.projects, refresh_s=self.config.graph_refresh_seconds or None)
        self.git = GitClient(self.config.git_clone_base_path, self.config.git_ssh_key_path,
                             self.config.git_timeout_seconds)
        self.backend = backend if backend is not None else create_backend(self.config)
        self.indexer = Indexer(self.repos, self.cache, self.git, self.backend,
                               batch_size=self.config.enrich_batch_size,
                               max_readme_length=self.config.max_readme_length,
                               description_length=self.config.description_length,
                               parser_threads=self.config.parser_threads,
                               require_enrichment=self.config.require_enrichment_for_analyze,
                               max_source_chars=self.config.enrich_max_source_chars,
                               in_memory_sources=self.config.git_in_memory,
                               in_memory_max_bytes=self.config.git_in_memory_max_mb << 20,
                               lease_ttl_s=self.config.project_lease_seconds,
                               stream_enrichment=self.config.enrich_stream,
                               scan_isolation=self.config.scan_isolation,
                               scan_timeout_s=self.config.scan_timeout_seconds)
        self.projects = ProjectService(self.repos, self.cache)
        self.context = ContextService(self.repos, self.cache)
        self.graph_query = GraphQueryService(self.cache)
        self._scheduler = None
        if self.config.recover_stuck_on_start:
            self.recover_stuck_projects()
        if load_graphs:
            self.cache.load_all()
        tune_gc()  # start-up heap out of the cyclic GC (see dmcp/utils/runtime.py)

    def recover_stuck_projects(self) -> int:
        """A project left ANALYZING/SYNCING by a dead process is moved to ERROR
        (the reference leaves it unrecoverable).  Only projects
        whose lease is free or expired: a live operation of another process
        (the analysis service while this MCP server starts) keeps its status."""
        import time as _time
        n = 0
        now = _time.time()
        for status in (ProjectStatus.ANALYZING, ProjectStatus.SYNCING):
            for p in self.repos.projects.find_by_status(status):
                owner, until = self.repos.projects.lease_of(p.id)
                if owner is not None and until is not None and float(until) >= now:
                    continue
                p.mark_error()
                self.repos.projects.update_status(p)
                n += 1
                LOG.warning("Recovered project %s stuck in %s -> ERROR", p.name, status.value)
        return n

    def start_scheduler(self) -> None:
        if not self.config.sync_enabled or self._scheduler is not None:
            return
        from .index.scheduler import CronScheduler
        self._scheduler = CronScheduler(self.config.sync_cron, self._scheduled_sync)
        self._scheduler.start()

    def _scheduled_sync(self) -> None:
        LOG.info("Starting scheduled project sync")
        r = self.indexer.sync_all_projects()
        LOG.info("Scheduled sync complete. Success: %d, Failed: %d", r.success_count, r.failure_count)

    def close(self) -> None:
        if self._scheduler is not None:
            self._scheduler.stop()
        self.backend.close()
        self.db.close()


_lock = threading.Lock()
