"""Indexing pipeline: analyze, rebuild-graph, incremental sync, resume.

Parity:

* :meth:`Indexer.analyze_project` -- ``CodeContextService.analyzeProject``
  (``:146-469``): READ_ONLY_MODE guard, RepositoryUrl validation, project
  create/reuse, shallow clone, README -> description (first 500 chars),
  parser detection, graph build, **Phase 1** static persist (classes, methods,
  parameter links), **Phase 2** enrichment in batches of 20 with at most 5
  concurrent calls, **Phase 3** recovery of ``description IS NULL`` classes
  when ``fixMissed``, graph JSON persisted, cache updated, endpoint count.
* :meth:`Indexer.rebuild_graph` -- ``CodeContextService.rebuildGraph`` (``:492-609``).
* :meth:`Indexer.sync_project` / :meth:`sync_all_projects` --
  ``ProjectSyncService`` (``:140-486``, ``:919-965``).
* :meth:`Indexer.apply_enrichment` -- ``CodeContextService.applyEnrichment`` (``:621-700``).

Fixes of documented reference defects:

* old data is replaced inside **one transaction after** clone+parse succeed
  (the reference deletes first, ``:745``, so a failed re-analysis lost data);
* sync has the Go branch (``ProjectSyncService.java:782-790`` lacked it);
* sync / rebuild graphs carry node + method metadata from the database, so
  ``graph_query`` no longer loses class types and descriptions after a sync;
* a project stuck in ANALYZING/SYNCING by a dead process is recovered to
  ERROR instead of being permanently wedged; per-project locks serialize
  analyze/sync of the same project inside this process;
* each phase runs in an explicit transaction (the reference's
  ``@Transactional`` on self-invoked methods never applied).
"""
from __future__ import annotations

import json
import logging
import os
import threading
import time
from concurrent.futures import TimeoutError as FutureTimeout
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

from ..enrich.backend import EnrichmentBackend, NullBackend, is_synthetic
from ..enrich.types import EnrichmentInput, EnrichmentResult, SizedIter, normalize_method_name
from ..graph.cache import GraphCache
from ..graph.project_graph import MethodEnrichmentData, MethodInfo, ProjectGraph
from ..models.domain import (ClassType, Project, ProjectStatus, RepositoryUrl, SourceClass,
                             new_id, new_ids, package_name_of, simple_name_of, utc_now)
from ..parsers.base import ParsedProject, ParsedUnit, SourceParser, parser_for
from ..store.repositories import ProjectRowsWriter, Repositories, to_iso
from ..utils.errors import DomainError
from ..utils.runtime import GcPause
from ..utils.tracing import METRICS, span
from .git import GitClient
from .lease import ProjectLease
from .source import CheckoutTree, SourceTree

LOG = logging.getLogger(__name__)


@dataclass
class AnalysisResult:
    success: bool
    project_id: Optional[str]
    classes_analyzed: int
    endpoints_found: int
    message: str
    stats: Dict[str, float] = field(default_factory=dict)

    def to_dict(self) -> dict:
        return {"success": self.success, "projectId": self.project_id,
                "classesAnalyzed": self.classes_analyzed, "endpointsFound": self.endpoints_found,
                "message": self.message}


@dataclass
class SyncResult:
    success: bool
    project_name: str
    commit_hash: Optional[str] = None
    added_classes: int = 0
    updated_classes: int = 0
    deleted_classes: int = 0
    unchanged_classes: int = 0
    enriched_classes: int = 0
    enrich_failed_classes: int = 0
    error_message: Optional[str] = None

    @classmethod
    def no_changes(cls, name: str) -> "SyncResult":
        return cls(True, name)

    @classmethod
    def failure(cls, name: str, msg: str) -> "SyncResult":
        return cls(False, name, error_message=msg)

    def to_dict(self) -> dict:
        return {"success": self.success, "projectName": self.project_name, "commitHash": self.commit_hash,
                "addedClasses": self.added_classes, "updatedClasses": self.updated_classes,
                "deletedClasses": self.deleted_classes, "unchangedClasses": self.unchanged_classes,
                "enrichedClasses": self.enriched_classes, "enrichFailedClasses": self.enrich_failed_classes,
                "errorMessage": self.error_message}


@dataclass
class SyncAllResult:
    success: bool
    total_projects: int
    success_count: int
    failure_count: int
    results: List[SyncResult]


def common_package_prefix(packages: Iterable[Optional[str]]) -> Optional[str]:
    """Longest common dotted prefix (CodeContextService.java:1752-1791)."""
    prefix: Optional[List[str]] = None
    seen_any = False
    for p in packages:
        if p is None:
            continue
        seen_any = True
        parts = p.split(".")
        if prefix is None:
            prefix = parts
            continue
        n = 0
        for a, b in zip(prefix, parts):
            if a != b:
                break
            n += 1
        prefix = prefix[:n]
    if not seen_any:
        return None
    return ".".join(prefix or [])


class _ProjectLocks:
    def __init__(self) -> None:
        self._locks: Dict[str, threading.Lock] = {}
        self._guard = threading.Lock()

    def get(self, key: str) -> threading.Lock:
        with self._guard:
            lk = self._locks.get(key)
            if lk is None:
                lk = self._locks[key] = threading.Lock()
            return lk


class Indexer:
    ROW_CHUNK = 256  # classes (with their methods) per writer put in Phase 1
    native_phase1 = True  # Phase 1 rows built by the native writer when it can (else the Python loop)
    phase1_ids: Optional[List[str]] = None  # row ids for the native Phase 1 (None = fresh UUIDv7s; tests)
    # a local repository's row swap opens before its snapshot read finishes
    # (the old rows' deletes overlap the read) and is rolled back if the read
    # is still running after this many seconds; a remote clone's opens after
    early_swap_wait_s = float(os.environ.get("DMCP_EARLY_SWAP_WAIT_S", "0.1"))

    def __init__(self, repos: Repositories, cache: GraphCache, git: GitClient,
                 backend: Optional[EnrichmentBackend] = None, *, batch_size: int = 20,
                 max_readme_length: int = 10_000, description_length: int = 500,
                 parser_threads: int = 0, require_enrichment: bool = True,
                 max_source_chars: int = 200_000, in_memory_sources: bool = True,
                 in_memory_max_bytes: int = 1 << 30, lease_ttl_s: float = 60.0,
                 stream_enrichment: bool = True, scan_isolation: str = "auto",
                 scan_timeout_s: float = 120.0) -> None:
        self.scan_isolation = (scan_isolation or "auto").lower()
        self.scan_timeout_s = scan_timeout_s
        self.lease_ttl_s = lease_ttl_s
        self.stream_enrichment = stream_enrichment
        self.in_memory_sources = in_memory_sources
        self.in_memory_max_bytes = in_memory_max_bytes
        self.repos = repos
        self.cache = cache
        self.git = git
        self.backend = backend or NullBackend(1)
        self.batch_size = max(1, int(batch_size))
        self.max_readme_length = max_readme_length
        self.description_length = description_length
        self.parser_threads = parser_threads
        self.require_enrichment = require_enrichment
        self.max_source_chars = max_source_chars
        self._locks = _ProjectLocks()
        self._io_pool = None  # snapshot reads that overlap the project-row preparation
        self._io_guard = threading.Lock()

    # ================================================================ analyze
    def analyze_project(self, repository_url: str, branch: Optional[str] = None,
                        fix_missed: bool = True) -> AnalysisResult:
        # automatic GC passes are held off from the parse on (GcPause,
        # dmcp/utils/runtime.py); without Phase 2 they resume only after the
        # analysis' frame is gone, when reference counting has freed its
        # parse objects and the previous graph: in steady state nothing is
        # left for a pass to scan.  With enrichment they resume before Phase 2.
        gcp = GcPause()
        try:
            return self._analyze(repository_url, branch, fix_missed, gcp)
        finally:
            gcp.resume()

    def _analyze(self, repository_url: str, branch: Optional[str], fix_missed: bool,
                 gcp: GcPause) -> AnalysisResult:
        if self.require_enrichment and not self.backend.enabled:
            # a refused backend (ENRICH_BACKEND=local without a checkpoint)
            # says why; otherwise the reference's message
            msg = getattr(self.backend, "disabled_reason", None) or \
                "Cannot run analysis in read-only mode. ANTHROPIC_API_KEY is not configured."
            LOG.error("%s", msg)
            raise DomainError(msg, "READ_ONLY_MODE")
        url = RepositoryUrl.of(repository_url)
        branch_name = branch if branch is not None else "main"
        lock = self._locks.get(url.value)
        if not lock.acquire(blocking=False):
            raise DomainError(f"Project {url.repository_name()} is already being processed",
                              "PROJECT_BUSY")
        stats: Dict[str, float] = {}
        clone: Optional[SourceTree] = None
        writer: Optional[ProjectRowsWriter] = None
        # the snapshot is read (natively, mostly without the GIL) on a helper
        # thread while the project row is looked up and marked ANALYZING
        fetch = self._submit_io(self._timed_fetch, url, branch_name)
        try:
            with span("analyze.prepare", stats):
                project, lease = self._prepare_project(url, branch_name)
        except BaseException:
            self._discard_fetch(fetch)
            lock.release()  # a failed status write must not leave the repository locked
            raise
        try:
            with span("analyze.total", stats, project=project.name):
                # the row swap's transaction (SQLite: BEGIN IMMEDIATE, the
                # database's write lock) must not be held across a slow read --
                # a remote clone can take far longer than other writers' busy
                # timeout -- so it opens after the snapshot is read, except for
                # a local repository, whose read is usually a few ms of
                # in-place object inflation: there it opens right away (the old
                # rows' deletes overlap the read) and is rolled back if the read
                # outlasts early_swap_wait_s.  The deletes run on the writer
                # thread while the tree is parsed (rolled back if it fails).
                with span("analyze.clone", stats):  # what is left of the read after the above
                    if self.early_swap_wait_s > 0 and url.local_path() is not None:
                        writer = self.repos.project_rows_writer(project.id, True)
                        try:
                            clone, stats["analyze.fetch"] = fetch.result(timeout=self.early_swap_wait_s)
                        except FutureTimeout:
                            writer.abort()  # a slow disk: release the write lock during the read
                            writer = None
                    if clone is None:
                        clone, stats["analyze.fetch"] = fetch.result()
                if writer is None:
                    writer = self.repos.project_rows_writer(project.id, True)
                readme = clone.readme(self.max_readme_length)
                if readme is not None:
                    project.update_description(readme[:self.description_length])
                parser = parser_for(clone.detect_language(), self.parser_threads)
                now = to_iso(utc_now())
                # the native scan hands the class / method rows to the writer
                # as soon as it has them (fresh UUIDv7s; not with given test ids)
                rows = (writer.static_rows(now, clone.commit_hash)
                        if self.native_phase1 and self.phase1_ids is None
                        and (not self._isolate(url) or self._iso_rows(clone)) else None)
                gcp.start()
                with span("analyze.parse", stats):
                    parsed = self._scan(parser, clone, url, rows=rows)
                    for k, v in (getattr(parsed, "scan_timing", None) or {}).items():
                        stats[f"analyze.parse_{k[:-3]}"] = v  # child / decode / objects (ms)
                    graph = parsed.build_graph()
                LOG.info("Graph built: %d nodes, %d entry points", graph.node_count(), graph.entry_point_count())
                order = graph.analysis_order()
                with span("analyze.phase1", stats):
                    # the swap stays open: it commits only under a live lease
                    # (without enrichment the project row joins it below)
                    p1 = self._phase1_static(project, parsed, graph, order, clone.commit_hash, writer,
                                             close=False, now=now)
                classes, methods_by_ident, writer = p1
                enriched = failed = recovered = 0
                if self.backend.enabled:
                    with span("analyze.phase1_commit", stats):
                        lease.check()  # never swap rows in over an operation that took the project over
                        writer.close()
                        gcp.resume(collect=True)  # a young pass, if due, under the writer's work
                        writer.wait()  # enrichment updates the rows just written
                    with span("analyze.phase2", stats):
                        enriched, failed = self._enrich_identifiers(order, parsed, graph, clone,
                                                                    readme, methods_by_ident, lease=lease)
                    if fix_missed:
                        with span("analyze.phase3", stats):
                            recovered = self._recover_unenriched(project, parsed, graph, clone, readme,
                                                                 lease=lease)
                lease.check()  # never publish over an operation that took the project over
                with span("analyze.persist_graph", stats):  # the graph JSON + the project row
                    project.base_package = common_package_prefix({package_name_of(i) for i in parsed.units})
                    project.update_graph_data(graph.to_json())
                    project.analysis_completed(clone.commit_hash)
                    # the version this write will give the row (read under the
                    # lease, before the write: the cache never pairs a newer
                    # version with this graph)
                    v0 = self.repos.projects.graph_version(project.id)
                    # the project row joins the row swap's transaction when the
                    # swap is still open (no enrichment), else it follows it
                    in_swap = writer.put_project_update(project)
                    if not writer.closed:
                        writer.close()
                # the row swap's writer thread (rows, then the commit) is the
                # analysis' critical path: this is the main thread's wait for it
                with span("analyze.phase1_commit", stats):
                    writer.wait()  # no-op when enrichment already waited
                for k, v in writer.timings.items():
                    if k.endswith("_ms"):  # (the *_s entries are absolute milestones)
                        stats[f"analyze.writer_{k[:-3]}"] = v
                with span("analyze.publish", stats):
                    if not in_swap:
                        self.repos.projects.update(project)
                    self.cache.put(project.id, project.name, graph, None if v0 is None else v0 + 1)
                endpoints = self.repos.methods.count_endpoints_by_project_id(project.id)
            METRICS.inc("classes_indexed", classes)
            LOG.info("Analysis completed. Classes: %d, Endpoints: %d, Enriched: %d, Enrich failed: %d, "
                     "Recovered: %d, timings(ms): %s", classes, endpoints, enriched, failed, recovered,
                     {k: round(v, 1) for k, v in stats.items()})
            stats.update({"classes": classes, "enriched": enriched, "enrichFailed": failed,
                          "recovered": recovered})
            return AnalysisResult(True, project.id, classes, endpoints, "Analysis complete", stats)
        except Exception as e:
            LOG.error("Analysis failed for %s: %s", repository_url, e, exc_info=True)
            if writer is not None:
                try:
                    writer.finish()  # the row swap ends (commit or rollback) before the status write
                except Exception:
                    pass
            if not lease.is_lost(e):  # a lost lease: the project's status is the new owner's
                self._mark_error(project)
            raise DomainError(f"Analysis failed: {e}", "ANALYSIS_FAILED", e) from e
        finally:
            with span("analyze.cleanup", stats):
                if clone is not None:
                    clone.cleanup()
            with span("analyze.release", stats):  # the lease row's release (one write)
                lease.release()
            lock.release()

    def _isolate(self, url: RepositoryUrl) -> Optional[float]:
        """Scan time limit when the scan must run in a child process: remote
        repositories under "auto" (untrusted input; the reference likewise
        ran its native analyzer out of process, GoSourceParser.java:339-418)."""
        if self.scan_isolation == "process" or (self.scan_isolation == "auto" and url.local_path() is None):
            return self.scan_timeout_s
        return None

    def _scan(self, parser: SourceParser, tree: SourceTree, url: RepositoryUrl, rows=None) -> ParsedProject:
        iso = self._isolate(url)
        return parser.scan_tree(tree, rows=rows if (not iso or self._iso_rows(tree)) else None,
                                isolate_timeout_s=iso)

    @staticmethod
    def _iso_rows(tree: SourceTree) -> bool:
        """An isolated scan of ``tree`` can hand its rows to the writer (the
        persistent binary child on an in-memory snapshot)."""
        from ..parsers import isolated
        return not isinstance(tree, CheckoutTree) and isolated.objects_supported()

    def _submit_io(self, fn, *args):
        with self._io_guard:
            if self._io_pool is None:
                from concurrent.futures import ThreadPoolExecutor
                self._io_pool = ThreadPoolExecutor(max_workers=4, thread_name_prefix="dmcp-fetch")
            return self._io_pool.submit(fn, *args)

    def _timed_fetch(self, url: RepositoryUrl, branch: Optional[str]) -> Tuple[SourceTree, float]:
        t0 = time.perf_counter()
        tree = self._fetch(url, branch, shallow=True)
        return tree, (time.perf_counter() - t0) * 1e3

    @staticmethod
    def _discard_fetch(fut) -> None:
        """An analysis that fails before it takes the snapshot: wait for the
        read and drop its tree (nothing else owns it)."""
        try:
            tree, _ = fut.result()
        except BaseException:
            return
        tree.cleanup()

    def _fetch(self, url: RepositoryUrl, branch: Optional[str], shallow: bool) -> SourceTree:
        """The branch head: in memory from git objects (default) or checked out."""
        if self.in_memory_sources:
            return self.git.snapshot(url, branch, shallow=shallow, max_bytes=self.in_memory_max_bytes)
        c = self.git.clone(url, branch, shallow=shallow)
        return CheckoutTree(c.directory, c.commit_hash)

    def analyze_local(self, path: str, fix_missed: bool = True) -> AnalysisResult:
        """Analyzes a local git working tree (``file://`` clone of HEAD)."""
        return self.analyze_project(os.path.abspath(path), branch=None, fix_missed=fix_missed)

    def _lease(self, project: Project) -> ProjectLease:
        """Takes the project's cross-process lease (``PROJECT_BUSY`` if held)."""
        return ProjectLease(self.repos.projects, project.id, self.lease_ttl_s, project.name).acquire()

    def _prepare_project(self, url: RepositoryUrl, branch: str) -> Tuple[Project, ProjectLease]:
        # the old graph is never read: a successful analysis replaces it, a
        # failed one only writes the status
        project = self.repos.projects.find_by_repository_url(url, with_graph=False)
        if project is None:
            project = Project.create(url.repository_name(), url, branch)
            try:
                self.repos.projects.save(project)
                LOG.info("Created new project: %s", project.id)
            except Exception:
                # another process registered the repository first (UNIQUE repository_url)
                project = self.repos.projects.find_by_repository_url(url, with_graph=False)
                if project is None:
                    raise
        lease = self._lease(project)
        try:
            # the status as the previous holder left it, read under the lease
            project = self.repos.projects.find_by_repository_url(url, with_graph=False) or project
            if project.status.is_processing():
                # we hold the lease, so that holder's lease ran out: it died
                LOG.warning("Project %s was left in %s by a process that stopped; recovering",
                            project.name, project.status.value)
                project.mark_error()
            project.default_branch = branch
            project.start_analysis()
            self.repos.projects.update_status(project)
        except BaseException:
            lease.release()
            raise
        return project, lease

    def _mark_error(self, project: Project) -> None:
        try:
            project.mark_error()
            self.repos.projects.update_status(project)
        except Exception as e:  # never mask the original failure
            LOG.warning("Could not mark project %s as ERROR: %s", project.id, e)

    # ---------------------------------------------------------------- phase 1
    def _phase1_static(self, project: Project, parsed: ParsedProject, graph: ProjectGraph,
                       order: Sequence[str], commit_hash: str, writer: Optional[ProjectRowsWriter] = None,
                       replace: bool = True, close: bool = True,
                       now: Optional[str] = None) -> Tuple[int, Dict[str, List[Tuple[str, str]]], ProjectRowsWriter]:
        """Builds every class / method / parameter row and the graph metadata
        and streams them to a :class:`ProjectRowsWriter` (``writer``, already
        started by the caller, or a new one), which swaps them in with one
        transaction (old rows deleted in it) on its own thread; the caller
        must ``wait()`` on the returned writer before touching the rows
        (and ``close()`` it first when ``close`` is False)."""
        now = now or to_iso(utc_now())
        pid = project.id
        cls_rows: List[tuple] = []
        meth_rows: List[tuple] = []
        param_rows: List[tuple] = []
        methods_by_ident: Dict[str, List[Tuple[str, str]]] = {}
        units = parsed.units
        class_ids: Dict[str, str] = {}
        if writer is None:  # the writer thread starts deleting the old rows right away
            writer = self.repos.project_rows_writer(pid, replace)
        if writer.native_phase1 and self.native_phase1:
            try:
                n_cls, n_meth, n_par, _, _, _, methods_by_ident, _ = writer.phase1_rows(
                    list(order), units, self.phase1_ids, now, commit_hash, MethodInfo, self.ROW_CHUNK,
                    graph.static_metadata_targets(), pre_ids=parsed.static_row_ids)
                if close:
                    writer.close()
            except BaseException:
                writer.abort()
                raise
            LOG.info("Phase 1 rows built natively. Classes: %d, Methods: %d, Parameters: %d", n_cls, n_meth, n_par)
            return n_cls, methods_by_ident, writer
        if parsed.static_row_ids is not None:  # those rows are already queued on a native writer
            raise RuntimeError("Phase 1: rows pre-written by the scan need the native Phase 1")
        # an upper bound of the ids needed: one per class and method, one per
        # parameter link of every method (overloads included)
        n_ids = 0
        for u in units.values():
            n_ids += 1 + len(u.methods)
            if u.params:
                n_ids += sum(len(u.params.get(m[0]) or ()) for m in u.methods)
        nid = iter(new_ids(n_ids)).__next__
        try:
            class_types: Dict[str, Optional[str]] = {}
            method_infos: Dict[str, List[MethodInfo]] = {}
            cls_append, meth_append = cls_rows.append, meth_rows.append
            dumps = json.dumps
            tnew, MI = tuple.__new__, MethodInfo  # NamedTuple without the generated __new__ wrapper
            # rows go to the writer in chunks, so its inserts overlap the
            # building of the rest (methods follow their classes' chunk)
            n_cls = n_meth = 0
            pending, chunk = 0, self.ROW_CHUNK
            for ident in order:
                unit = units.get(ident)
                if unit is None:
                    continue
                if pending == chunk:
                    writer.put("classes", cls_rows)
                    writer.put("methods", meth_rows)
                    n_cls, n_meth = n_cls + len(cls_rows), n_meth + len(meth_rows)
                    cls_rows, meth_rows = [], []
                    cls_append, meth_append = cls_rows.append, meth_rows.append
                    pending = 0
                pending += 1
                cid = nid()
                class_ids[ident] = cid
                ct = unit.class_type.value
                i = ident.rfind(".")
                cls_append((cid, pid, ident, ident[i + 1:] if i >= 0 else ident,
                            ident[:i] if i >= 0 else None, ct, None, unit.source_file, now, commit_hash))
                class_types[ident] = ct
                infos = []
                mids = []
                for name, line, http_method, http_path, exc in unit.methods:
                    mid = nid()
                    meth_append((mid, cid, name, None, "[]", dumps(list(exc)) if exc else "[]", http_method,
                                 http_path, line, now))
                    infos.append(tnew(MI, (name, None, (), exc, http_method, http_path, line)))
                    mids.append((name, mid))
                method_infos[ident] = infos
                methods_by_ident[ident] = mids
            writer.put("classes", cls_rows)
            writer.put("methods", meth_rows)
            n_cls, n_meth = n_cls + len(cls_rows), n_meth + len(meth_rows)
            # parameter links (CodeContextService.java:274-291, 805-856): the
            # first method of each name that has resolved parameter types
            links: Dict[str, Dict[str, List[str]]] = {}
            for ident, mids in methods_by_ident.items():
                params = units[ident].params
                if not params or not mids:
                    continue
                per: Dict[str, List[str]] = {}
                for mname, mid in mids:
                    targets = params.get(mname)
                    if not targets:
                        continue
                    if mname not in per:
                        per[mname] = targets
                    for pos, tgt in enumerate(targets):
                        tcid = class_ids.get(tgt)
                        if tcid is not None:
                            param_rows.append((nid(), mid, pos, tcid, now))
                if per:
                    links[ident] = per
            writer.put("params", param_rows)
            graph.load_static_metadata(class_ids, class_types, method_infos, links)
            if close:
                writer.close()
        except BaseException:
            writer.abort()
            raise
        LOG.info("Phase 1 rows built. Classes: %d, Methods: %d, Parameters: %d", n_cls, n_meth, len(param_rows))
        return n_cls, methods_by_ident, writer

    # ------------------------------------------------------------ enrichment
    def _read_source(self, tree: SourceTree, unit: ParsedUnit) -> Optional[str]:
        parts = []
        total = 0
        for rel in (unit.files if len(unit.files) > 1 else [unit.source_file]):
            text = tree.read_text(rel)
            if text is None:
                LOG.warning("Failed to read source for enrichment %s", rel)
                continue
            if len(unit.files) > 1:
                text = f"// file: {rel}\n{text}"
            parts.append(text)
            total += len(text)
            if self.max_source_chars and total >= self.max_source_chars:
                break
        return "\n".join(parts) if parts else None

    def _inputs_for(self, idents: Sequence[str], parsed: ParsedProject, tree: SourceTree,
                    class_types: Optional[Dict[str, str]] = None) -> Tuple[List[EnrichmentInput], int]:
        inputs, failed = [], 0
        for ident in idents:
            unit = parsed.units.get(ident)
            if unit is None:
                continue
            src = self._read_source(tree, unit)
            if src is None:
                failed += 1
                continue
            ct = (class_types or {}).get(ident, unit.class_type.value)
            inputs.append(EnrichmentInput(src, ident, parsed.language, ct,
                                          [m.method_name for m in unit.methods]))
        return inputs, failed

    def _input_for(self, ident: str, parsed: ParsedProject, tree: SourceTree,
                   class_types: Optional[Dict[str, str]] = None) -> Optional[EnrichmentInput]:
        unit = parsed.units.get(ident)
        if unit is None:
            return None
        src = self._read_source(tree, unit)
        if src is None:
            return None
        ct = (class_types or {}).get(ident, unit.class_type.value)
        return EnrichmentInput(src, ident, parsed.language, ct, [m.method_name for m in unit.methods])

    def _stream_enrich(self, idents: Sequence[str], parsed: ParsedProject, graph: ProjectGraph,
                       tree: SourceTree, readme: Optional[str], class_types: Optional[Dict[str, str]],
                       methods_by_ident: Optional[Dict[str, List[Tuple[str, str]]]], phase: str,
                       lease: Optional[ProjectLease] = None) -> Tuple[int, int]:
        """Every pending class goes to the backend as ONE stream (sources read
        lazily, as the backend asks for more); each result is applied the
        moment it arrives.  A local GPU engine keeps its continuous batch full
        across the whole project; API backends keep ``max_concurrent`` in
        flight (a sliding window, not 20-class barriers)."""
        read_failed = [0]
        total = len(idents)
        pending = [i for i in idents if i in parsed.units]

        def gen():
            for ident in pending:
                inp = self._input_for(ident, parsed, tree, class_types)
                if inp is None:
                    read_failed[0] += 1
                    continue
                yield inp
        enriched = failed = 0
        step = max(20, total // 10)
        # lazy, but sized: a multi-GPU backend deals ceil(pending / GPUs) per GPU
        inputs = SizedIter(gen(), len(pending))
        for n, (_, result) in enumerate(self.backend.enrich_stream(inputs, readme), 1):
            if lease is not None:
                lease.check()  # every write: once the lease ran out the rows may be another owner's
            if not result.success:
                LOG.warning("%s: enrichment failed for %s: %s", phase, result.full_class_name, result.error_message)
                failed += 1
            elif self.apply_enrichment(result, graph, methods_by_ident):
                enriched += 1
            else:
                failed += 1
            if n % step == 0:
                LOG.info("%s: %d/%d classes enriched (%d failed)", phase, enriched, total, failed)
        return enriched, failed + read_failed[0]

    def _enrich_identifiers(self, idents: Sequence[str], parsed: ParsedProject, graph: ProjectGraph,
                            tree: SourceTree, readme: Optional[str],
                            methods_by_ident: Optional[Dict[str, List[Tuple[str, str]]]] = None,
                            lease: Optional[ProjectLease] = None) -> Tuple[int, int]:
        idents = list(idents)
        if self.stream_enrichment:
            enriched, failed = self._stream_enrich(idents, parsed, graph, tree, readme, None, methods_by_ident,
                                                   "Phase 2", lease)
        else:  # the reference's barriers: batches of batch_size classes (CodeContextService.java:297-359)
            enriched = failed = 0
            nbatches = (len(idents) + self.batch_size - 1) // self.batch_size
            for b in range(0, len(idents), self.batch_size):
                batch = idents[b:b + self.batch_size]
                LOG.info("Enriching batch %d/%d (%d classes)", b // self.batch_size + 1, nbatches, len(batch))
                inputs, read_failed = self._inputs_for(batch, parsed, tree)
                failed += read_failed
                if lease is not None:
                    lease.check()
                for result in self.backend.enrich_batch(inputs, readme):
                    if not result.success:
                        LOG.warning("Enrichment failed for %s: %s", result.full_class_name, result.error_message)
                        failed += 1
                        continue
                    self.apply_enrichment(result, graph, methods_by_ident)
                    enriched += 1
        METRICS.inc("classes_enriched", enriched)
        METRICS.inc("classes_enrich_failed", failed)
        return enriched, failed

    def _recover_unenriched(self, project: Project, parsed: ParsedProject, graph: ProjectGraph,
                            tree: SourceTree, readme: Optional[str], lease: Optional[ProjectLease] = None) -> int:
        # a real backend also redoes what a synthetic one (random weights,
        # fake, echo) wrote; a synthetic backend redoes only missing rows
        unenriched = self.repos.classes.find_unenriched_by_project_id(
            project.id, include_synthetic=not is_synthetic(self.backend.source_tag))
        if not unenriched:
            LOG.info("Phase 3: No unenriched classes found, skipping recovery")
            return 0
        LOG.info("Phase 3: Found %d classes with missing enrichment, retrying", len(unenriched))
        types = {sc.full_class_name: sc.class_type.value for sc in unenriched}
        idents = [sc.full_class_name for sc in unenriched]
        if self.stream_enrichment:
            recovered, _ = self._stream_enrich(idents, parsed, graph, tree, readme, types, None, "Phase 3", lease)
        else:
            recovered = 0
            for b in range(0, len(idents), self.batch_size):
                inputs, _ = self._inputs_for(idents[b:b + self.batch_size], parsed, tree, types)
                if not inputs:
                    continue
                for result in self.backend.enrich_batch(inputs, readme):
                    if result.success:
                        self.apply_enrichment(result, graph)
                        recovered += 1
                    else:
                        LOG.warning("Phase 3: Recovery failed for %s: %s", result.full_class_name,
                                    result.error_message)
        LOG.info("Phase 3 complete. Recovered: %d/%d", recovered, len(unenriched))
        return recovered

    def apply_enrichment(self, result: EnrichmentResult, graph: ProjectGraph,
                         methods_by_ident: Optional[Dict[str, List[Tuple[str, str]]]] = None) -> bool:
        """Writes one class's enrichment to the DB and the (unpublished) graph."""
        fqcn = result.full_class_name
        class_id = graph.class_id(fqcn)
        if class_id is None:
            LOG.warning("No classId found for %s during enrichment", fqcn)
            return False
        correction: Optional[ClassType] = None
        c = result.class_type_correction
        if c is not None and c.strip() and c.strip().lower() != "null":
            name = c.strip().upper()
            if name in ClassType.__members__:
                correction = ClassType[name]
        # method name -> first method id (by extraction order == line order)
        if methods_by_ident is not None and fqcn in methods_by_ident:
            name_to_id: Dict[str, str] = {}
            for mname, mid in methods_by_ident[fqcn]:
                name_to_id.setdefault(mname, mid)
        else:
            name_to_id = {}
            for m in self.repos.methods.find_by_class_id(class_id):
                name_to_id.setdefault(m.method_name, m.id)
        updates = []
        enrichments: Dict[str, MethodEnrichmentData] = {}
        for me in result.methods:
            mname = normalize_method_name(me.method_name)
            mid = name_to_id.get(mname)
            if mid is None:
                LOG.debug("Method %s not found for enrichment in class %s", mname, fqcn)
                continue
            updates.append((me.description, list(me.business_logic), mid))
            enrichments[mname] = MethodEnrichmentData(me.description, tuple(me.business_logic))
        tag = self.backend.source_tag
        with self.repos.db.transaction() as conn:
            if correction is not None:
                conn.execute("UPDATE source_classes SET class_type = ?, description = ?, enrichment_source = ? "
                             "WHERE id = ?", (correction.value, result.description, tag, class_id))
            else:
                conn.execute("UPDATE source_classes SET description = ?, enrichment_source = ? WHERE id = ?",
                             (result.description, tag, class_id))
            self.repos.methods.update_enrichment_batch(updates)
        if correction is not None:
            resolved = correction.value
        else:
            ni = graph.node_info(fqcn)
            resolved = ni.class_type if ni is not None and ni.class_type else "OTHER"
        if not graph.frozen:
            graph.apply_enrichment(fqcn, resolved, result.description, enrichments)
        return True

    # ================================================================ rebuild
    def rebuild_graph(self, project_id: str) -> dict:
        project = self.repos.projects.find_by_id(project_id)
        if project is None:
            raise DomainError(f"Project not found: {project_id}", "PROJECT_NOT_FOUND")
        lock = self._locks.get(project.repository_url.value)
        if not lock.acquire(blocking=False):
            raise DomainError(f"Project {project.name} is already being processed", "PROJECT_BUSY")
        try:
            lease = self._lease(project)
        except BaseException:
            lock.release()
            raise
        clone = None
        stats: Dict[str, float] = {}
        try:
            with span("rebuild.total", stats, project=project.name):
                clone = self._fetch(project.repository_url, project.default_branch, shallow=True)
                parser = parser_for(clone.detect_language(), self.parser_threads)
                parsed = self._scan(parser, clone, project.repository_url)
                graph = parsed.build_graph()
                existing = self.repos.classes.find_by_project_id(project_id)
                by_name = {sc.full_class_name: sc for sc in existing}
                bound = 0
                for ident in graph.identifiers():
                    sc = by_name.get(ident)
                    if sc is not None:
                        graph.bind_class_id(ident, sc.id)
                        bound += 1
                LOG.info("Rebuild: bound %d/%d identifiers", bound, graph.node_count())
                missing_hash = [sc.id for sc in existing if sc.commit_hash is None]
                self.repos.classes.update_commit_hash_batch(missing_hash, clone.commit_hash)
                methods_by_class = self.repos.methods.find_by_class_ids([sc.id for sc in existing])
                self._attach_metadata(graph, parsed, by_name, methods_by_class)
                param_rows = self._param_rows(graph, parsed, by_name, methods_by_class)
                with self.repos.db.transaction():
                    self.repos.params.delete_by_project_id(project_id)
                    self.repos.params.save_rows(param_rows)
                project.update_graph_data(graph.to_json())
                project.base_package = common_package_prefix({package_name_of(i) for i in parsed.units})
                lease.check()
                self.repos.projects.update(project)
                self.cache.put(project_id, project.name, graph)
            return {"success": True, "projectId": project_id, "bound": bound,
                    "parameters": len(param_rows), "stats": stats}
        except DomainError:
            raise
        except Exception as e:
            LOG.error("Graph rebuild failed for %s: %s", project_id, e, exc_info=True)
            raise DomainError(f"Graph rebuild failed: {e}", "REBUILD_FAILED", e) from e
        finally:
            if clone is not None:
                clone.cleanup()
            lease.release()
            lock.release()

    def _attach_metadata(self, graph: ProjectGraph, parsed: ParsedProject, by_name: Dict[str, SourceClass],
                         methods_by_class: Dict[str, list]) -> None:
        """Node/method metadata for a freshly parsed graph: persisted enrichment
        where a row exists, static facts otherwise (fixes SURVEY §3.5)."""
        for ident, unit in parsed.units.items():
            sc = by_name.get(ident)
            if sc is not None:
                graph.set_node_info(ident, sc.class_type.value, sc.description)
                rows = methods_by_class.get(sc.id) or []
                graph.set_method_infos(ident, [
                    MethodInfo(m.method_name, m.description, tuple(m.business_logic), tuple(m.exceptions),
                               m.http_method, m.http_path, m.line_number) for m in rows])
            else:
                graph.set_node_info(ident, unit.class_type.value, None)
                graph.set_method_infos(ident, [
                    MethodInfo(sm.method_name, None, (), tuple(sm.exceptions), sm.http_method, sm.http_path,
                               sm.line_number) for sm in unit.methods])

    def _param_rows(self, graph: ProjectGraph, parsed: ParsedProject, by_name: Dict[str, SourceClass],
                    methods_by_class: Dict[str, list], only: Optional[Iterable[str]] = None) -> List[tuple]:
        now = to_iso(utc_now())
        rows: List[tuple] = []
        idents = list(only) if only is not None else list(parsed.units)
        for ident in idents:
            unit = parsed.units.get(ident)
            sc = by_name.get(ident)
            if unit is None or sc is None or not unit.params:
                continue
            graph.clear_method_parameters(ident)
            linked = set()
            for m in methods_by_class.get(sc.id) or []:
                targets = unit.params.get(m.method_name)
                if not targets:
                    continue
                if m.method_name not in linked:
                    linked.add(m.method_name)
                    for pos, tgt in enumerate(targets):
                        graph.add_method_parameter(ident, m.method_name, pos, tgt)
                for pos, tgt in enumerate(targets):
                    tcid = graph.class_id(tgt)
                    if tcid is not None:
                        rows.append((new_id(), m.id, pos, tcid, now))
        return rows

    # =================================================================== sync
    def sync_project(self, project: Project) -> SyncResult:
        lock = self._locks.get(project.repository_url.value)
        if not lock.acquire(blocking=False):
            return SyncResult.failure(project.name, "project is already being processed")
        try:
            lease = self._lease(project)
        except DomainError:
            lock.release()
            return SyncResult.failure(project.name, "project is already being processed")
        except BaseException:
            lock.release()
            raise
        clone = None
        stats: Dict[str, float] = {}
        try:
            project = self.repos.projects.find_by_id(project.id) or project  # state under the lease
            if project.status.is_processing():
                project.mark_error()  # we hold the lease: the process that left it there stopped
            project.start_sync()
            self.repos.projects.update_status(project)
            with span("sync.total", stats, project=project.name):
                # full history: the diff needs the previously analyzed commit
                clone = self._fetch(project.repository_url, project.default_branch, shallow=False)
                head = clone.commit_hash
                if head == project.last_commit_hash:
                    LOG.info("No changes detected for project: %s (HEAD: %s)", project.name, head)
                    project.sync_completed(project.last_commit_hash)
                    self.repos.projects.update_status(project)
                    return SyncResult.no_changes(project.name)
                diff = self.git.diff(clone.git_dir, project.last_commit_hash, head)
                readme = clone.readme(self.max_readme_length)
                if readme is not None:
                    project.update_description(readme[:self.description_length])
                parser = parser_for(clone.detect_language(), self.parser_threads)
                parsed = self._scan(parser, clone, project.repository_url)
                graph = parsed.build_graph()
                existing = self.repos.classes.find_by_project_id(project.id)
                by_name = {sc.full_class_name: sc for sc in existing}
                new_ids = parsed.units
                to_delete = [n for n in by_name if n not in new_ids]
                to_add, to_update, unchanged = [], [], []
                for ident, unit in new_ids.items():
                    if ident not in by_name:
                        to_add.append(ident)
                    elif diff.full_resync_required or any(f in diff.changed_files for f in unit.files):
                        to_update.append(ident)
                    else:
                        unchanged.append(ident)
                LOG.info("Changes for %s: add=%d, update=%d, delete=%d, unchanged=%d", project.name,
                         len(to_add), len(to_update), len(to_delete), len(unchanged))
                now = to_iso(utc_now())
                cls_rows, meth_rows = [], []
                methods_by_ident: Dict[str, List[Tuple[str, str]]] = {}
                with self.repos.db.transaction() as conn:
                    if to_delete:
                        ids = [by_name[n].id for n in to_delete]
                        self.repos.params.delete_by_class_ids(ids)
                        self.repos.methods.delete_by_class_ids(ids)
                        self.repos.classes.delete_by_ids(ids)
                    # updated classes keep their row (and id); their methods and
                    # parameter links are replaced -- one statement per table for
                    # all of them, not N round trips (Postgres)
                    upd_ids = [by_name[i].id for i in to_update]
                    self.repos.params.delete_by_class_ids(upd_ids)
                    self.repos.methods.delete_by_class_ids(upd_ids)
                    conn.executemany("UPDATE source_classes SET commit_hash = ?, class_type = ?, source_file = ? "
                                     "WHERE id = ?", [(head, new_ids[i].class_type.value, new_ids[i].source_file,
                                                      by_name[i].id) for i in to_update])
                    for ident in to_update:
                        sc = by_name[ident]
                        unit = new_ids[ident]
                        graph.bind_class_id(ident, sc.id)
                        mids = []
                        for sm in unit.methods:
                            mid = new_id()
                            meth_rows.append((mid, sc.id, sm.method_name, None, "[]", json.dumps(list(sm.exceptions)),
                                              sm.http_method, sm.http_path, sm.line_number, now))
                            mids.append((sm.method_name, mid))
                        methods_by_ident[ident] = mids
                    for ident in to_add:
                        unit = new_ids[ident]
                        cid = new_id()
                        cls_rows.append((cid, project.id, ident, simple_name_of(ident), package_name_of(ident),
                                         unit.class_type.value, None, unit.source_file, now, head))
                        graph.bind_class_id(ident, cid)
                        mids = []
                        for sm in unit.methods:
                            mid = new_id()
                            meth_rows.append((mid, cid, sm.method_name, None, "[]", json.dumps(list(sm.exceptions)),
                                              sm.http_method, sm.http_path, sm.line_number, now))
                            mids.append((sm.method_name, mid))
                        methods_by_ident[ident] = mids
                    for ident in unchanged:
                        graph.bind_class_id(ident, by_name[ident].id)
                    self.repos.classes.save_rows(cls_rows)
                    self.repos.methods.save_rows(meth_rows)
                # parameter links for changed classes; unchanged ones keep their rows
                all_classes = {sc.full_class_name: sc for sc in self.repos.classes.find_by_project_id(project.id)}
                changed = to_add + to_update
                mb = self.repos.methods.find_by_class_ids([all_classes[i].id for i in changed if i in all_classes])
                param_rows = self._param_rows(graph, parsed, all_classes, mb, only=changed)
                self.repos.params.save_rows(param_rows)
                # unchanged classes: rebuild their graph links from the parse as well
                mb_un = self.repos.methods.find_by_class_ids([all_classes[i].id for i in unchanged if i in all_classes])
                self._relink_graph_only(graph, parsed, all_classes, mb_un, unchanged)
                enriched = failed = 0
                if self.backend.enabled and changed:
                    self._attach_metadata(graph, parsed, all_classes, {**mb_un, **mb})
                    enriched, failed = self._enrich_identifiers(changed, parsed, graph, clone, readme,
                                                                methods_by_ident, lease=lease)
                # final metadata from the DB (enrichment included)
                final_classes = {sc.full_class_name: sc for sc in self.repos.classes.find_by_project_id(project.id)}
                mb_all = self.repos.methods.find_by_class_ids([sc.id for sc in final_classes.values()])
                self._attach_metadata(graph, parsed, final_classes, mb_all)
                project.base_package = common_package_prefix({package_name_of(i) for i in parsed.units})
                project.update_graph_data(graph.to_json())
                project.sync_completed(head)
                lease.check()
                self.repos.projects.update(project)
                self.cache.put(project.id, project.name, graph)
            LOG.info("Sync completed for %s. Added: %d, Updated: %d, Deleted: %d, Unchanged: %d, Enriched: %d, "
                     "EnrichFailed: %d", project.name, len(to_add), len(to_update), len(to_delete),
                     len(unchanged), enriched, failed)
            return SyncResult(True, project.name, head, len(to_add), len(to_update), len(to_delete),
                              len(unchanged), enriched, failed, None)
        except Exception as e:
            LOG.error("Sync failed for %s: %s", project.name, e, exc_info=True)
            if not lease.is_lost(e):  # a lost lease: the project's status is the new owner's
                self._mark_error(project)
            return SyncResult.failure(project.name, str(e))
        finally:
            if clone is not None:
                clone.cleanup()
            lease.release()
            lock.release()

    def _relink_graph_only(self, graph: ProjectGraph, parsed: ParsedProject, classes: Dict[str, SourceClass],
                           methods_by_class: Dict[str, list], idents: Iterable[str]) -> None:
        for ident in idents:
            unit = parsed.units.get(ident)
            sc = classes.get(ident)
            if unit is None or sc is None or not unit.params:
                continue
            linked = set()
            for m in methods_by_class.get(sc.id) or []:
                targets = unit.params.get(m.method_name)
                if targets and m.method_name not in linked:
                    linked.add(m.method_name)
                    for pos, tgt in enumerate(targets):
                        graph.add_method_parameter(ident, m.method_name, pos, tgt)

    def sync_all_projects(self) -> SyncAllResult:
        projects = self.repos.projects.find_by_statuses([ProjectStatus.ANALYZED, ProjectStatus.ERROR])
        if not projects:
            LOG.info("No projects eligible for sync")
            return SyncAllResult(True, 0, 0, 0, [])
        results: List[SyncResult] = []
        ok = bad = 0
        for p in projects:
            try:
                r = self.sync_project(p)
            except Exception as e:  # pragma: no cover - sync_project never raises
                r = SyncResult.failure(p.name, str(e))
            results.append(r)
            if r.success:
                ok += 1
            else:
                bad += 1
        LOG.info("Sync complete. Success: %d, Failed: %d", ok, bad)
        return SyncAllResult(bad == 0, len(projects), ok, bad, results)

    # ================================================================= resume
    def resume_enrichment(self, project_id: str) -> dict:
        """Checkpoint/resume: re-enriches every ``description IS NULL`` class of an
        analyzed project without re-running the static phase."""
        project = self.repos.projects.find_by_id(project_id)
        if project is None:
            raise DomainError(f"Project not found: {project_id}", "PROJECT_NOT_FOUND")
        if not self.backend.enabled:
            raise DomainError(getattr(self.backend, "disabled_reason", None) or "No enrichment backend configured",
                              "READ_ONLY_MODE")
        lock = self._locks.get(project.repository_url.value)
        if not lock.acquire(blocking=False):
            raise DomainError(f"Project {project.name} is already being processed", "PROJECT_BUSY")
        clone = None
        try:
            # resume writes enrichment onto the project's rows: it must not
            # race an analyze / sync that is replacing them (same lease)
            with self._lease(project) as lease:
                project = self.repos.projects.find_by_id(project_id) or project
                cached = self.cache.get_graph(project_id)
                graph = cached.copy() if cached is not None else (
                    ProjectGraph.from_json(project.graph_data) if project.graph_data else None)
                if graph is None:
                    raise DomainError("No graph data available for this project", "NO_GRAPH")
                clone = self._fetch(project.repository_url, project.default_branch, shallow=True)
                parsed = self._scan(parser_for(clone.detect_language(), self.parser_threads), clone,
                                    project.repository_url)
                readme = clone.readme(self.max_readme_length)
                recovered = self._recover_unenriched(project, parsed, graph, clone, readme, lease=lease)
                project.update_graph_data(graph.to_json())
                lease.check()
                self.repos.projects.update(project)
                self.cache.put(project.id, project.name, graph)
                return {"success": True, "projectId": project_id, "recovered": recovered}
        finally:
            if clone is not None:
                clone.cleanup()
            lock.release()
