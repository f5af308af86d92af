"""Repositories: SQL CRUD over the four tables.

Parity (reference SQL constants are quoted in each docstring):

* :class:`ProjectRepository`         -- ``project/domain/ProjectRepository.java:24-281``
* :class:`SourceClassRepository`     -- ``analysis/domain/SourceClassRepository.java:24-388``
* :class:`SourceMethodRepository`    -- ``analysis/domain/SourceMethodRepository.java:28-403``
* :class:`MethodParameterRepository` -- ``analysis/domain/MethodParameterRepository.java:27-179``

Divergences:

* ``find_by_full_class_name`` no longer throws when a FQCN exists in several
  projects (JDBI ``findOne`` at ``SourceClassRepository.java:171-177``); it
  returns the row of the most recently analyzed project.  ``find_all_by_full_class_name``
  exposes every match.
* ``find_by_class_name_and_method_name`` no longer throws on overloads
  (``SourceMethodRepository.java:206-214``); it returns the first overload by
  line number.
* batch ``*_in`` finders replace the per-row N+1 lookups of the context ops.
"""
from __future__ import annotations

import json
from datetime import datetime, timezone
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

from ..models.domain import (ClassType, MethodParameter, Project, ProjectStatus,
                             RepositoryUrl, SourceClass, SourceMethod)
from ..utils.errors import DomainError
from .db import Database

_CHUNK = 500  # SQLite host-parameter limit is 999 on older builds


def to_iso(dt: Optional[datetime]) -> Optional[str]:
    if dt is None:
        return None
    if dt.tzinfo is None:
        dt = dt.replace(tzinfo=timezone.utc)
    return dt.astimezone(timezone.utc).strftime("%Y-%m-%dT%H:%M:%S.%fZ")


def from_iso(s: Optional[str]) -> Optional[datetime]:
    if not s:
        return None
    s = s.strip()
    if s.endswith("Z"):
        s = s[:-1] + "+00:00"
    try:
        dt = datetime.fromisoformat(s)
    except ValueError:
        return None
    if dt.tzinfo is None:
        dt = dt.replace(tzinfo=timezone.utc)
    return dt


def _chunks(seq: Sequence, n: int = _CHUNK):
    for i in range(0, len(seq), n):
        yield seq[i:i + n]


def _json_list(value: Optional[Iterable[str]]) -> str:
    return json.dumps(list(value or ()), ensure_ascii=False)


def _parse_json_list(text: Optional[str]) -> List[str]:
    if not text or text == "[]":  # the common case: no exceptions / no logic
        return []
    try:
        v = json.loads(text)
    except ValueError:
        return []
    if isinstance(v, list):
        return [str(x) for x in v]
    return []


# --------------------------------------------------------------------------
class ProjectRepository:
    FIND_BY_ID = "SELECT * FROM projects WHERE id = ?"
    FIND_BY_REPOSITORY_URL = "SELECT * FROM projects WHERE repository_url = ?"
    FIND_BY_NAME = "SELECT * FROM projects WHERE name = ? ORDER BY created_at DESC LIMIT 1"
    FIND_ALL = "SELECT * FROM projects ORDER BY created_at DESC"
    FIND_BY_STATUS = "SELECT * FROM projects WHERE status = ?"
    FIND_ALL_WITH_GRAPH = "SELECT * FROM projects WHERE graph_data IS NOT NULL"
    EXISTS_BY_REPOSITORY_URL = "SELECT COUNT(*) FROM projects WHERE repository_url = ?"

    # columns without graph_data: list views never load the (large) graph JSON
    _LIGHT_COLUMNS = ("id, name, repository_url, default_branch, status, last_analyzed_at, "
                      "last_commit_hash, created_at, updated_at, description, base_package, "
                      "NULL AS graph_data")

    # SQLite (``db.graph_table``, migration 9): the graph JSON in its own
    # table, so a status or lease write never rewrites it -- every statement
    # above that returns graph_data reads it through this join
    _SPLIT_SELECT = ("SELECT p.id, p.name, p.repository_url, p.default_branch, p.status, p.last_analyzed_at, "
                     "p.last_commit_hash, p.created_at, p.updated_at, p.description, p.base_package, "
                     "g.graph_data AS graph_data FROM projects p {join} project_graphs g ON g.project_id = p.id")
    UPSERT_GRAPH = ("INSERT INTO project_graphs (project_id, graph_data) VALUES (?, ?) "
                    "ON CONFLICT (project_id) DO UPDATE SET graph_data = excluded.graph_data")
    DELETE_GRAPH = "DELETE FROM project_graphs WHERE project_id = ?"
    UPDATE_SPLIT = ("UPDATE projects SET name=?, default_branch=?, status=?, last_analyzed_at=?, "
                    "last_commit_hash=?, updated_at=?, description=?, base_package=?, "
                    "graph_version = graph_version + 1 WHERE id=?")

    def __init__(self, db: Database) -> None:
        self.db = db
        self.split = bool(getattr(db, "graph_table", False))
        if self.split:
            sel = self._SPLIT_SELECT.format(join="LEFT JOIN")
            self.FIND_BY_ID = f"{sel} WHERE p.id = ?"
            self.FIND_BY_REPOSITORY_URL = f"{sel} WHERE p.repository_url = ?"
            self.FIND_BY_NAME = f"{sel} WHERE p.name = ? ORDER BY p.created_at DESC LIMIT 1"
            self.FIND_ALL = f"{sel} ORDER BY p.created_at DESC"
            self.FIND_BY_STATUS = f"{sel} WHERE p.status = ?"
            self.FIND_ALL_WITH_GRAPH = self._SPLIT_SELECT.format(join="JOIN")

    @staticmethod
    def _map(row) -> Project:
        return Project.reconstitute(
            row["id"], row["name"], RepositoryUrl.of(row["repository_url"]),
            row["default_branch"], row["description"], ProjectStatus(row["status"]),
            from_iso(row["last_analyzed_at"]), row["last_commit_hash"], row["graph_data"],
            from_iso(row["created_at"]), from_iso(row["updated_at"]), row["base_package"])

    def save(self, p: Project) -> None:
        with self.db.transaction() as c:
            c.execute(
                "INSERT INTO projects (id, name, repository_url, default_branch, status, "
                "last_analyzed_at, last_commit_hash, created_at, updated_at, description, "
                "graph_data, base_package) VALUES (?,?,?,?,?,?,?,?,?,?,?,?)",
                (p.id, p.name, p.repository_url.value, p.default_branch, p.status.value,
                 to_iso(p.last_analyzed_at), p.last_commit_hash, to_iso(p.created_at),
                 to_iso(p.updated_at), p.description, None if self.split else p.graph_data, p.base_package))
            if self.split and p.graph_data is not None:
                c.execute(self.UPSERT_GRAPH, (p.id, p.graph_data))

    # a full update replaces the graph: its version moves, so the graph cache
    # of every other process reloads it (GraphCache.refresh)
    UPDATE = ("UPDATE projects SET name=?, default_branch=?, status=?, last_analyzed_at=?, "
              "last_commit_hash=?, updated_at=?, description=?, graph_data=?, base_package=?, "
              "graph_version = graph_version + 1 WHERE id=?")

    # -------------------------------------------------------------- lease
    # One operation (analyze / sync / rebuild / resume) per project across
    # every process sharing the database: the lease is taken with ONE
    # conditional upsert (atomic under SQLite's write lock and PostgreSQL's
    # row lock), heartbeated while the operation runs and released at its
    # end.  A crashed holder stops heartbeating, so its lease expires and the
    # next operation takes over (the reference's state machine instead
    # wedged a crashed ANALYZING project forever, ProjectStateMachine.java:34-70).
    # The lease has its own table (migration V8): SQLite rewrites a whole row
    # on any UPDATE, and the projects row carries the multi-megabyte graph
    # JSON -- three lease writes per analysis on that row cost ~17 % of it.
    ACQUIRE_LEASE = ("INSERT INTO project_leases (project_id, lease_owner, lease_until) VALUES (?, ?, ?) "
                     "ON CONFLICT (project_id) DO UPDATE SET lease_owner = excluded.lease_owner, "
                     "lease_until = excluded.lease_until "
                     "WHERE project_leases.lease_until < ? OR project_leases.lease_owner = excluded.lease_owner")
    RENEW_LEASE = "UPDATE project_leases SET lease_until = ? WHERE project_id = ? AND lease_owner = ?"
    RELEASE_LEASE = "DELETE FROM project_leases WHERE project_id = ? AND lease_owner = ?"

    def try_acquire_lease(self, project_id: str, owner: str, ttl_s: float, now: float) -> bool:
        with self.db.transaction() as c:
            cur = c.execute(self.ACQUIRE_LEASE, (project_id, owner, now + ttl_s, now))
            return cur.rowcount == 1

    def renew_lease(self, project_id: str, owner: str, until: float) -> bool:
        with self.db.transaction() as c:
            return c.execute(self.RENEW_LEASE, (until, project_id, owner)).rowcount == 1

    def release_lease(self, project_id: str, owner: str) -> bool:
        with self.db.transaction() as c:
            return c.execute(self.RELEASE_LEASE, (project_id, owner)).rowcount == 1

    def lease_of(self, project_id: str) -> Tuple[Optional[str], Optional[float]]:
        row = self.db.query_one("SELECT lease_owner, lease_until FROM project_leases WHERE project_id = ?",
                                (project_id,))
        return (row["lease_owner"], row["lease_until"]) if row else (None, None)

    def graph_versions(self) -> Dict[str, Tuple[str, int]]:
        """id -> (name, graph version) of every project with a persisted graph
        (one index-free scan of the small projects table; no graph JSON read)."""
        rows = self.db.query("SELECT p.id AS id, p.name AS name, p.graph_version AS graph_version FROM projects p "
                             "JOIN project_graphs g ON g.project_id = p.id" if self.split else
                             "SELECT id, name, graph_version FROM projects WHERE graph_data IS NOT NULL")
        return {r["id"]: (r["name"], int(r["graph_version"] or 0)) for r in rows}

    def graph_version(self, project_id: str) -> Optional[int]:
        row = self.db.query_one("SELECT graph_version FROM projects WHERE id = ?", (project_id,))
        return int(row["graph_version"] or 0) if row else None

    @staticmethod
    def update_params(p: Project) -> tuple:
        return (p.name, p.default_branch, p.status.value, to_iso(p.last_analyzed_at),
                p.last_commit_hash, to_iso(p.updated_at), p.description, p.graph_data,
                p.base_package, p.id)

    def update_statements(self, p: Project) -> List[Tuple[str, tuple]]:
        """The full update of ``p`` as (sql, params) statements of one
        transaction (the graph's own row on SQLite)."""
        if not self.split:
            return [(self.UPDATE, self.update_params(p))]
        row = (p.name, p.default_branch, p.status.value, to_iso(p.last_analyzed_at), p.last_commit_hash,
               to_iso(p.updated_at), p.description, p.base_package, p.id)
        graph = (self.UPSERT_GRAPH, (p.id, p.graph_data)) if p.graph_data is not None else \
            (self.DELETE_GRAPH, (p.id,))
        return [(self.UPDATE_SPLIT, row), graph]

    def update(self, p: Project) -> None:
        with self.db.transaction() as c:
            for sql, params in self.update_statements(p):
                c.execute(sql, params)

    def update_status(self, p: Project) -> None:
        """Status-only update that does not rewrite the graph column."""
        with self.db.transaction() as c:
            c.execute("UPDATE projects SET status=?, updated_at=?, last_analyzed_at=?, "
                      "last_commit_hash=?, description=? WHERE id=?",
                      (p.status.value, to_iso(p.updated_at), to_iso(p.last_analyzed_at),
                       p.last_commit_hash, p.description, p.id))

    def find_by_id(self, project_id: str) -> Optional[Project]:
        row = self.db.query_one(self.FIND_BY_ID, (project_id,))
        return self._map(row) if row else None

    def find_by_repository_url(self, url, with_graph: bool = True) -> Optional[Project]:
        """``with_graph=False``: graph_data is not read (None) -- for callers
        that replace it anyway (a re-analysis), the JSON is megabytes."""
        value = url.value if isinstance(url, RepositoryUrl) else str(url)
        q = (self.FIND_BY_REPOSITORY_URL if with_graph
             else f"SELECT {self._LIGHT_COLUMNS} FROM projects WHERE repository_url = ?")
        row = self.db.query_one(q, (value,))
        return self._map(row) if row else None

    def find_by_name(self, name: str) -> Optional[Project]:
        row = self.db.query_one(self.FIND_BY_NAME, (name,))
        return self._map(row) if row else None

    def find_all(self, with_graph: bool = False) -> List[Project]:
        if with_graph:
            return [self._map(r) for r in self.db.query(self.FIND_ALL)]
        rows = self.db.query(f"SELECT {self._LIGHT_COLUMNS} FROM projects ORDER BY created_at DESC")
        return [self._map(r) for r in rows]

    def find_by_status(self, status: ProjectStatus) -> List[Project]:
        return [self._map(r) for r in self.db.query(self.FIND_BY_STATUS, (status.value,))]

    def find_by_statuses(self, statuses: Iterable[ProjectStatus]) -> List[Project]:
        vals = [s.value for s in statuses]
        if not vals:
            return []
        marks = ','.join('?' * len(vals))
        q = (f"{self._SPLIT_SELECT.format(join='LEFT JOIN')} WHERE p.status IN ({marks}) ORDER BY p.created_at"
             if self.split else f"SELECT * FROM projects WHERE status IN ({marks}) ORDER BY created_at")
        return [self._map(r) for r in self.db.query(q, vals)]

    def find_all_with_graph(self) -> List[Project]:
        return [self._map(r) for r in self.db.query(self.FIND_ALL_WITH_GRAPH)]

    def delete(self, project_id: str) -> None:
        with self.db.transaction() as c:
            c.execute("DELETE FROM projects WHERE id = ?", (project_id,))

    def exists_by_repository_url(self, url) -> bool:
        value = url.value if isinstance(url, RepositoryUrl) else str(url)
        row = self.db.query_one(self.EXISTS_BY_REPOSITORY_URL, (value,))
        return bool(row[0])


# --------------------------------------------------------------------------
class SourceClassRepository:
    FIND_BY_ID = "SELECT * FROM source_classes WHERE id = ?"
    FIND_BY_PROJECT_ID = "SELECT * FROM source_classes WHERE project_id = ? ORDER BY full_class_name"
    FIND_BY_FULL_CLASS_NAME = (
        "SELECT c.* FROM source_classes c JOIN projects p ON p.id = c.project_id "
        "WHERE c.full_class_name = ? "
        "ORDER BY p.last_analyzed_at DESC NULLS LAST, p.created_at DESC")
    # range form of "package_name LIKE 'p.%'" (what text_pattern_ops gives the
    # reference on Postgres): SQLite only uses an index for LIKE under
    # case_sensitive_like, a range always can
    FIND_BY_PACKAGE_PREFIX = ("SELECT * FROM source_classes WHERE package_name = ? "
                              "OR (package_name >= ? AND package_name < ?) ORDER BY full_class_name")
    COUNT_BY_PROJECT_ID = "SELECT COUNT(*) FROM source_classes WHERE project_id = ?"
    FIND_BY_PROJECT_ID_AND_FULL_CLASS_NAME = (
        "SELECT * FROM source_classes WHERE project_id = ? AND full_class_name = ?")
    FIND_UNENRICHED_BY_PROJECT_ID = ("SELECT * FROM source_classes WHERE project_id = ? "
                                     "AND description IS NULL ORDER BY full_class_name")
    # ... plus the rows a synthetic backend enriched (migration 10)
    FIND_UNENRICHED_OR_SYNTHETIC_BY_PROJECT_ID = (
        "SELECT * FROM source_classes WHERE project_id = ? "
        "AND (description IS NULL OR enrichment_source LIKE 'synthetic:%') ORDER BY full_class_name")
    _INSERT = ("INSERT INTO source_classes (id, project_id, full_class_name, simple_name, "
               "package_name, class_type, description, source_file, created_at, commit_hash) "
               "VALUES (?,?,?,?,?,?,?,?,?,?)")

    def __init__(self, db: Database) -> None:
        self.db = db

    @staticmethod
    def _map(row) -> SourceClass:
        return SourceClass(row["id"], row["project_id"], row["full_class_name"], row["simple_name"],
                           row["package_name"], ClassType.from_string(row["class_type"]),
                           row["description"], row["source_file"], row["commit_hash"],
                           from_iso(row["created_at"]))

    @staticmethod
    def _params(sc: SourceClass):
        return (sc.id, sc.project_id, sc.full_class_name, sc.simple_name, sc.package_name,
                sc.class_type.value, sc.description, sc.source_file, to_iso(sc.created_at),
                sc.commit_hash)

    def save(self, sc: SourceClass) -> None:
        with self.db.transaction() as c:
            c.execute(self._INSERT, self._params(sc))

    def save_all(self, classes: Sequence[SourceClass]) -> None:
        if not classes:
            return
        with self.db.transaction() as c:
            c.executemany(self._INSERT, [self._params(sc) for sc in classes])

    def save_rows(self, rows: Sequence[tuple]) -> None:
        """Bulk insert of pre-built parameter tuples (hot indexing path)."""
        if not rows:
            return
        with self.db.transaction() as c:
            c.executemany(self._INSERT, rows)

    def find_by_id(self, class_id: str) -> Optional[SourceClass]:
        row = self.db.query_one(self.FIND_BY_ID, (class_id,))
        return self._map(row) if row else None

    def find_by_ids(self, ids: Sequence[str]) -> Dict[str, SourceClass]:
        out: Dict[str, SourceClass] = {}
        for chunk in _chunks(list(ids)):
            q = f"SELECT * FROM source_classes WHERE id IN ({','.join('?' * len(chunk))})"
            for r in self.db.query(q, chunk):
                out[r["id"]] = self._map(r)
        return out

    def find_by_project_id(self, project_id: str) -> List[SourceClass]:
        return [self._map(r) for r in self.db.query(self.FIND_BY_PROJECT_ID, (project_id,))]

    def find_by_full_class_name(self, fqcn: str) -> Optional[SourceClass]:
        row = self.db.query_one(self.FIND_BY_FULL_CLASS_NAME, (fqcn,))
        return self._map(row) if row else None

    def find_all_by_full_class_name(self, fqcn: str) -> List[SourceClass]:
        return [self._map(r) for r in self.db.query(self.FIND_BY_FULL_CLASS_NAME, (fqcn,))]

    def find_by_full_class_names(self, names: Sequence[str],
                                 project_id: Optional[str] = None) -> Dict[str, SourceClass]:
        """Batch lookup: FQCN -> class (first by most recent project, like the single form)."""
        out: Dict[str, SourceClass] = {}
        uniq = list(dict.fromkeys(n for n in names if n is not None))
        for chunk in _chunks(uniq):
            marks = ",".join("?" * len(chunk))
            if project_id is not None:
                q = (f"SELECT * FROM source_classes WHERE project_id = ? "
                     f"AND full_class_name IN ({marks})")
                rows = self.db.query(q, [project_id, *chunk])
            else:
                q = (f"SELECT c.* FROM source_classes c JOIN projects p ON p.id = c.project_id "
                     f"WHERE c.full_class_name IN ({marks}) "
                     f"ORDER BY p.last_analyzed_at DESC NULLS LAST, p.created_at DESC")
                rows = self.db.query(q, chunk)
            for r in rows:
                if r["full_class_name"] not in out:
                    out[r["full_class_name"]] = self._map(r)
        return out

    def find_by_package_prefix(self, package_prefix: str) -> List[SourceClass]:
        # "p" or "p.*" as two index ranges: [p, p] and [p + ".", p + "/") ('/' follows '.')
        return [self._map(r) for r in self.db.query(self.FIND_BY_PACKAGE_PREFIX,
                                                    (package_prefix, package_prefix + ".", package_prefix + "/"))]

    def find_by_project_id_and_full_class_name(self, project_id: str, fqcn: str) -> Optional[SourceClass]:
        row = self.db.query_one(self.FIND_BY_PROJECT_ID_AND_FULL_CLASS_NAME, (project_id, fqcn))
        return self._map(row) if row else None

    def count_by_project_id(self, project_id: str) -> int:
        return int(self.db.query_one(self.COUNT_BY_PROJECT_ID, (project_id,))[0])

    def count_by_project(self) -> Dict[str, int]:
        return {r[0]: int(r[1]) for r in self.db.query(
            "SELECT project_id, COUNT(*) FROM source_classes GROUP BY project_id")}

    def class_type_breakdown(self, project_id: str) -> Dict[str, int]:
        return {r[0]: int(r[1]) for r in self.db.query(
            "SELECT class_type, COUNT(*) FROM source_classes WHERE project_id = ? "
            "GROUP BY class_type ORDER BY class_type", (project_id,))}

    def package_names(self, project_id: str) -> List[str]:
        return [r[0] for r in self.db.query(
            "SELECT DISTINCT package_name FROM source_classes WHERE project_id = ? "
            "AND package_name IS NOT NULL", (project_id,))]

    def update_enrichment(self, class_id: str, class_type: ClassType, description: Optional[str]) -> None:
        with self.db.transaction() as c:
            c.execute("UPDATE source_classes SET class_type = ?, description = ? WHERE id = ?",
                      (class_type.value, description, class_id))

    def update_description(self, class_id: str, description: Optional[str]) -> None:
        with self.db.transaction() as c:
            c.execute("UPDATE source_classes SET description = ? WHERE id = ?", (description, class_id))

    def update_commit_hash(self, class_id: str, commit_hash: Optional[str]) -> None:
        with self.db.transaction() as c:
            c.execute("UPDATE source_classes SET commit_hash = ? WHERE id = ?", (commit_hash, class_id))

    def update_commit_hash_batch(self, class_ids: Sequence[str], commit_hash: Optional[str]) -> None:
        if not class_ids:
            return
        with self.db.transaction() as c:
            c.executemany("UPDATE source_classes SET commit_hash = ? WHERE id = ?",
                          [(commit_hash, i) for i in class_ids])

    DELETE_BY_PROJECT_ID = "DELETE FROM source_classes WHERE project_id = ?"

    def delete_by_project_id(self, project_id: str) -> None:
        with self.db.transaction() as c:
            c.execute(self.DELETE_BY_PROJECT_ID, (project_id,))

    def delete_by_ids(self, ids: Sequence[str]) -> None:
        if not ids:
            return
        with self.db.transaction() as c:
            for chunk in _chunks(list(ids)):
                c.execute(f"DELETE FROM source_classes WHERE id IN ({','.join('?' * len(chunk))})",
                          chunk)

    def delete(self, class_id: str) -> None:
        """One class; its methods and parameter links go with it (FK cascade)."""
        with self.db.transaction() as c:
            c.execute("DELETE FROM source_classes WHERE id = ?", (class_id,))

    def find_unenriched_by_project_id(self, project_id: str, include_synthetic: bool = False) -> List[SourceClass]:
        """Classes without a description; with ``include_synthetic`` also the
        classes whose description a synthetic backend wrote (random weights,
        fake, echo: ``enrichment_source`` 'synthetic:...')."""
        q = self.FIND_UNENRICHED_OR_SYNTHETIC_BY_PROJECT_ID if include_synthetic else self.FIND_UNENRICHED_BY_PROJECT_ID
        return [self._map(r) for r in self.db.query(q, (project_id,))]

    def enrichment_sources(self, project_id: str) -> Dict[str, Optional[str]]:
        """full_class_name -> enrichment_source of a project's classes."""
        return {r[0]: r[1] for r in self.db.query(
            "SELECT full_class_name, enrichment_source FROM source_classes WHERE project_id = ?", (project_id,))}


# --------------------------------------------------------------------------
class SourceMethodRepository:
    FIND_BY_ID = "SELECT * FROM source_methods WHERE id = ?"
    FIND_BY_CLASS_ID = ("SELECT * FROM source_methods WHERE class_id = ? "
                        "ORDER BY line_number IS NULL, line_number, method_name")
    FIND_BY_CLASS_NAME = ("SELECT m.* FROM source_methods m JOIN source_classes c ON c.id = m.class_id "
                          "WHERE c.full_class_name = ? "
                          "ORDER BY m.line_number IS NULL, m.line_number, m.method_name")
    FIND_BY_CLASS_AND_METHOD_NAME = (
        "SELECT m.* FROM source_methods m JOIN source_classes c ON c.id = m.class_id "
        "WHERE c.full_class_name = ? AND m.method_name = ? "
        "ORDER BY m.line_number IS NULL, m.line_number")
    FIND_BY_CLASS_ID_AND_METHOD_NAME = (
        "SELECT * FROM source_methods WHERE class_id = ? AND method_name = ? "
        "ORDER BY line_number IS NULL, line_number LIMIT 1")
    FIND_HTTP_ENDPOINTS_BY_PROJECT_ID = (
        "SELECT m.* FROM source_methods m JOIN source_classes c ON c.id = m.class_id "
        "WHERE c.project_id = ? AND m.http_method IS NOT NULL AND m.http_path IS NOT NULL "
        "ORDER BY m.http_path, m.http_method")
    COUNT_ENDPOINTS_BY_PROJECT_ID = (
        "SELECT COUNT(*) FROM source_methods m JOIN source_classes c ON c.id = m.class_id "
        "WHERE c.project_id = ? AND m.http_method IS NOT NULL AND m.http_path IS NOT NULL")
    _INSERT = ("INSERT INTO source_methods (id, class_id, method_name, description, business_logic, "
               "exceptions, http_method, http_path, line_number, created_at) "
               "VALUES (?,?,?,?,?,?,?,?,?,?)")

    def __init__(self, db: Database) -> None:
        self.db = db

    @staticmethod
    def _map(row) -> SourceMethod:
        return SourceMethod(row["id"], row["class_id"], row["method_name"], row["description"],
                            _parse_json_list(row["business_logic"]), _parse_json_list(row["exceptions"]),
                            row["http_method"], row["http_path"], row["line_number"],
                            from_iso(row["created_at"]))

    @staticmethod
    def _params(m: SourceMethod):
        return (m.id, m.class_id, m.method_name, m.description, _json_list(m.business_logic),
                _json_list(m.exceptions), m.http_method, m.http_path, m.line_number,
                to_iso(m.created_at))

    def save(self, m: SourceMethod) -> None:
        with self.db.transaction() as c:
            c.execute(self._INSERT, self._params(m))

    def save_all(self, methods: Sequence[SourceMethod]) -> None:
        if not methods:
            return
        with self.db.transaction() as c:
            c.executemany(self._INSERT, [self._params(m) for m in methods])

    def save_rows(self, rows: Sequence[tuple]) -> None:
        if not rows:
            return
        with self.db.transaction() as c:
            c.executemany(self._INSERT, rows)

    def find_by_id(self, method_id: str) -> Optional[SourceMethod]:
        row = self.db.query_one(self.FIND_BY_ID, (method_id,))
        return self._map(row) if row else None

    def find_by_class_id(self, class_id: str) -> List[SourceMethod]:
        return [self._map(r) for r in self.db.query(self.FIND_BY_CLASS_ID, (class_id,))]

    def find_by_class_ids(self, class_ids: Sequence[str]) -> Dict[str, List[SourceMethod]]:
        out: Dict[str, List[SourceMethod]] = {cid: [] for cid in class_ids}
        for chunk in _chunks(list(dict.fromkeys(class_ids))):
            q = (f"SELECT * FROM source_methods WHERE class_id IN ({','.join('?' * len(chunk))}) "
                 f"ORDER BY line_number IS NULL, line_number, method_name")
            for r in self.db.query(q, chunk):
                out.setdefault(r["class_id"], []).append(self._map(r))
        return out

    def find_by_class_name(self, fqcn: str) -> List[SourceMethod]:
        return [self._map(r) for r in self.db.query(self.FIND_BY_CLASS_NAME, (fqcn,))]

    def find_by_class_name_and_method_name(self, fqcn: str, method_name: str) -> Optional[SourceMethod]:
        row = self.db.query_one(self.FIND_BY_CLASS_AND_METHOD_NAME, (fqcn, method_name))
        return self._map(row) if row else None

    def find_by_class_id_and_method_name(self, class_id: str, method_name: str) -> Optional[SourceMethod]:
        row = self.db.query_one(self.FIND_BY_CLASS_ID_AND_METHOD_NAME, (class_id, method_name))
        return self._map(row) if row else None

    def find_http_endpoints_by_project_id(self, project_id: str) -> List[SourceMethod]:
        return [self._map(r) for r in self.db.query(self.FIND_HTTP_ENDPOINTS_BY_PROJECT_ID, (project_id,))]

    def count_endpoints_by_project_id(self, project_id: str) -> int:
        return int(self.db.query_one(self.COUNT_ENDPOINTS_BY_PROJECT_ID, (project_id,))[0])

    def count_endpoints_by_project(self) -> Dict[str, int]:
        return {r[0]: int(r[1]) for r in self.db.query(
            "SELECT c.project_id, COUNT(*) FROM source_methods m JOIN source_classes c "
            "ON c.id = m.class_id WHERE m.http_method IS NOT NULL AND m.http_path IS NOT NULL "
            "GROUP BY c.project_id")}

    def update_enrichment(self, method_id: str, description: Optional[str],
                          business_logic: Optional[Iterable[str]],
                          exceptions: Optional[Iterable[str]]) -> None:
        with self.db.transaction() as c:
            c.execute("UPDATE source_methods SET description = ?, business_logic = ?, exceptions = ? "
                      "WHERE id = ?", (description, _json_list(business_logic),
                                       _json_list(exceptions), method_id))

    def update_enrichment_batch(self, rows: Sequence[tuple]) -> None:
        """rows: (description, business_logic_list, method_id)."""
        if not rows:
            return
        with self.db.transaction() as c:
            c.executemany("UPDATE source_methods SET description = ?, business_logic = ? WHERE id = ?",
                          [(d, _json_list(bl), mid) for d, bl, mid in rows])

    def delete_by_class_id(self, class_id: str) -> None:
        with self.db.transaction() as c:
            c.execute("DELETE FROM source_methods WHERE class_id = ?", (class_id,))

    def delete(self, method_id: str) -> None:
        with self.db.transaction() as c:
            c.execute("DELETE FROM source_methods WHERE id = ?", (method_id,))

    DELETE_BY_PROJECT_ID = ("DELETE FROM source_methods WHERE class_id IN "
                            "(SELECT id FROM source_classes WHERE project_id = ?)")

    def delete_by_project_id(self, project_id: str) -> None:
        with self.db.transaction() as c:
            c.execute(self.DELETE_BY_PROJECT_ID, (project_id,))

    def delete_by_class_ids(self, class_ids: Sequence[str]) -> None:
        if not class_ids:
            return
        with self.db.transaction() as c:
            for chunk in _chunks(list(class_ids)):
                c.execute(f"DELETE FROM source_methods WHERE class_id IN ({','.join('?' * len(chunk))})",
                          chunk)


# --------------------------------------------------------------------------
class MethodParameterRepository:
    FIND_BY_METHOD_ID = "SELECT * FROM method_parameters WHERE method_id = ? ORDER BY position"
    _INSERT = ("INSERT INTO method_parameters (id, method_id, position, class_id, created_at) "
               "VALUES (?,?,?,?,?)")

    def __init__(self, db: Database) -> None:
        self.db = db

    @staticmethod
    def _map(row) -> MethodParameter:
        return MethodParameter(row["id"], row["method_id"], int(row["position"]), row["class_id"],
                               from_iso(row["created_at"]))

    @staticmethod
    def _params(p: MethodParameter):
        return (p.id, p.method_id, p.position, p.class_id, to_iso(p.created_at))

    def save(self, p: MethodParameter) -> None:
        with self.db.transaction() as c:
            self._check_same_project(c, [(p.method_id, p.class_id)])
            c.execute(self._INSERT, self._params(p))

    def save_all(self, params: Sequence[MethodParameter]) -> None:
        if not params:
            return
        with self.db.transaction() as c:
            self._check_same_project(c, [(p.method_id, p.class_id) for p in params])
            c.executemany(self._INSERT, [self._params(p) for p in params])

    @staticmethod
    def _check_same_project(c, links: Sequence[Tuple[str, str]]) -> None:
        """Rejects a link whose method and parameter class live in different
        projects.  The project-scoped delete (:attr:`DELETE_BY_PROJECT_ID`)
        selects links by their target class only, which is exact only under
        this invariant; the analysis paths satisfy it by construction (targets
        are resolved among the project's own classes) and write through
        :meth:`save_rows`.  Unknown ids are left to the foreign keys."""
        method_ids = list({m for m, _ in links})
        class_ids = list({k for _, k in links})
        owner: Dict[str, str] = {}
        for chunk in _chunks(method_ids):
            for mid, pid in c.execute(
                    "SELECT m.id, k.project_id FROM source_methods m JOIN source_classes k ON k.id = m.class_id "
                    f"WHERE m.id IN ({','.join('?' * len(chunk))})", chunk):
                owner[mid] = pid
        target: Dict[str, str] = {}
        for chunk in _chunks(class_ids):
            for cid, pid in c.execute(
                    f"SELECT id, project_id FROM source_classes WHERE id IN ({','.join('?' * len(chunk))})", chunk):
                target[cid] = pid
        for mid, cid in links:
            a, b = owner.get(mid), target.get(cid)
            if a is not None and b is not None and a != b:
                raise DomainError(f"Method parameter links method {mid} (project {a}) to class {cid} "
                                  f"of another project ({b})", "PARAMETER_CROSS_PROJECT")

    def save_rows(self, rows: Sequence[tuple]) -> None:
        if not rows:
            return
        with self.db.transaction() as c:
            c.executemany(self._INSERT, rows)

    def find_by_method_id(self, method_id: str) -> List[MethodParameter]:
        return [self._map(r) for r in self.db.query(self.FIND_BY_METHOD_ID, (method_id,))]

    def delete_by_method_id(self, method_id: str) -> None:
        with self.db.transaction() as c:
            c.execute("DELETE FROM method_parameters WHERE method_id = ?", (method_id,))

    def delete_by_class_id(self, class_id: str) -> None:
        """Deletes every link whose parameter TYPE is ``class_id``
        (``MethodParameterRepository.java:127-133``: ``WHERE class_id = ?``)."""
        with self.db.transaction() as c:
            c.execute("DELETE FROM method_parameters WHERE class_id = ?", (class_id,))

    def delete_by_owner_class_id(self, class_id: str) -> None:
        """Deletes the parameter links of every method declared BY ``class_id``
        (the single-class form of :meth:`delete_by_class_ids`)."""
        with self.db.transaction() as c:
            c.execute("DELETE FROM method_parameters WHERE method_id IN "
                      "(SELECT id FROM source_methods WHERE class_id = ?)", (class_id,))

    def delete_by_class_ids(self, class_ids: Sequence[str]) -> None:
        if not class_ids:
            return
        with self.db.transaction() as c:
            for chunk in _chunks(list(class_ids)):
                c.execute("DELETE FROM method_parameters WHERE method_id IN (SELECT id FROM source_methods "
                          f"WHERE class_id IN ({','.join('?' * len(chunk))}))", chunk)

    # A parameter link always joins a method and a class of the SAME project
    # (targets are resolved among the project's own classes), so selecting the
    # links by their target class reaches exactly the project's links -- and
    # it is the set ON DELETE CASCADE of the classes would remove anyway.  Via
    # idx_method_params_class this visits one index range per class instead of
    # class -> methods -> links (2.5x cheaper on an 8,000-class project).
    DELETE_BY_PROJECT_ID = ("DELETE FROM method_parameters WHERE class_id IN "
                            "(SELECT id FROM source_classes WHERE project_id = ?)")

    def delete_by_project_id(self, project_id: str) -> None:
        with self.db.transaction() as c:
            c.execute(self.DELETE_BY_PROJECT_ID, (project_id,))


class Repositories:
    """Bundle of the four repositories over one database."""

    def __init__(self, db: Database) -> None:
        self.db = db
        self.projects = ProjectRepository(db)
        self.classes = SourceClassRepository(db)
        self.methods = SourceMethodRepository(db)
        self.params = MethodParameterRepository(db)

    def project_rows_writer(self, project_id: str, replace: bool) -> "ProjectRowsWriter":
        return ProjectRowsWriter(self, project_id, replace)


class ProjectRowsWriter:
    """Whole-project row swap (old class/method/parameter rows deleted, new
    ones inserted, one transaction) run on a writer thread while the caller
    is still building the rows.

    The reference saves rows one JPA/JDBI call at a time inside the analysis
    loop (``CodeContextService.java:244-291``).  Here the writer thread opens
    the transaction as soon as the writer is created (the indexer creates it
    before it reads and parses the snapshot) and deletes the project's old
    rows meanwhile; the caller then streams row chunks with :meth:`put` while
    it is still building the rest, and the thread inserts each chunk as it
    arrives.

    On a database file the writer is native (``native/srcscan/bulkwriter.cpp``):
    its own SQLite connection on a C++ thread, so binding and B-tree work run
    without the GIL and overlap the Python row building and the graph
    serialisation that follows (a Python writer thread would convoy on the GIL
    once per row).  Without the native module, a Python thread does the same
    work.  A private ``:memory:`` database (one shared connection) runs the
    steps synchronously.  :meth:`wait` re-raises any writer error;
    :meth:`abort` rolls the transaction back.
    """

    _TABLES = ("classes", "methods", "params")
    BUSY_TIMEOUT_MS = 30_000

    def __init__(self, repos: "Repositories", project_id: str, replace: bool) -> None:
        import queue
        import threading
        self.repos = repos
        self.project_id = project_id
        self.replace = replace
        self.rows_written = 0
        self.timings: Dict[str, float] = {}  # native writer phases (ms), after wait()
        self._error: Optional[BaseException] = None
        self._sync = repos.db.is_shared_memory()
        self._q: "queue.Queue" = queue.Queue()
        self._pending: List[Tuple[str, Sequence[tuple]]] = []
        self._thread: Optional[threading.Thread] = None
        self._done = False
        self._native = None
        # the native writer reads text straight out of these objects' UTF-8
        # buffers: they stay referenced here until its thread has finished
        self._keep: List[object] = []
        if self._sync:
            return
        bulk = _native_bulk_writer() if getattr(repos.db, "native_bulk", True) else None
        if bulk is not None:
            setup = []
            if getattr(repos.db, "checkpointer", None) is not None:
                # checkpoints belong to the database's background thread
                setup.append(("PRAGMA wal_autocheckpoint = 0", ((),)))
            if replace:
                setup += [(r.DELETE_BY_PROJECT_ID, ((project_id,),))
                          for r in (repos.params, repos.methods, repos.classes)]
            self._keep.append(setup)
            self._native = bulk(repos.db.path, self.BUSY_TIMEOUT_MS, setup)
            return
        self._thread = threading.Thread(target=self._run, name="dmcp-rows-writer", daemon=True)
        self._thread.start()

    # ------------------------------------------------------------ producer
    def put(self, table: str, rows: Sequence[tuple]) -> None:
        """Queues rows of one table; tables may be put repeatedly and
        interleaved (the producer streams chunks while it builds the rest),
        inserted in arrival order.  Foreign keys are not enforced during the
        swap (native writer / ``bulk_transaction``); a ``:memory:`` database
        keeps them on, so put each row after the rows it references."""
        if table not in self._TABLES:
            raise ValueError(f"unknown table {table}")
        if self._native is not None:
            if rows:
                frozen = tuple(rows)  # immutable: the writer holds views into it
                self._keep.append(frozen)
                self._native.put(getattr(self.repos, table)._INSERT, frozen)
        elif self._sync:
            self._pending.append((table, rows))
        else:
            self._q.put((table, rows))

    @property
    def closed(self) -> bool:
        """:meth:`close` was called (a commit is on its way)."""
        return getattr(self, "_closed", False)

    def finish(self) -> None:
        """Error-path cleanup: waits for a requested commit, rolls back otherwise
        (a writer that was never closed would wait for rows forever)."""
        if self.closed:
            self.wait()
        else:
            self.abort()

    @property
    def native_phase1(self) -> bool:
        """The native writer can build the Phase 1 rows itself (:meth:`phase1_rows`)."""
        return self._native is not None and hasattr(self._native, "phase1_rows")

    def phase1_rows(self, order, units, ids: Optional[list], now: str, commit_hash: Optional[str], method_info_cls,
                    chunk: int = 256, graph_targets: Optional[tuple] = None, pre_ids: Optional[dict] = None) -> tuple:
        """Class / method / parameter rows of the parsed ``units`` (in
        ``order``) built natively and streamed to this writer in ``chunk``-class
        batches -- the Python loop of ``Indexer._phase1_static`` without a
        tuple per row (``native/srcscan/pymodule.cpp::phase1_rows``).  ``ids``:
        the row ids to use in order, or None for fresh UUIDv7s.
        ``graph_targets`` (``ProjectGraph.static_metadata_targets()``): the
        graph's metadata is filled in place instead of returned.  Returns
        (n_classes, n_methods, n_params, class_ids, class_types, method_infos,
        methods_by_ident, links)."""
        self._keep.append((order, units, ids, now, commit_hash, pre_ids))  # the native rows are views into these
        r = self.repos
        out = self._native.phase1_rows(order, units, ids, self.project_id, now, commit_hash, r.classes._INSERT,
                                       r.methods._INSERT, r.params._INSERT, method_info_cls, chunk, graph_targets,
                                       pre_ids)
        self._keep.append(out[-1])  # ids generated natively
        return out[:-1]

    def static_rows(self, now: str, commit_hash: Optional[str]) -> Optional[tuple]:
        """What ``scan_sources_objects(rows=...)`` needs to write the class /
        method rows straight from the native scan into this writer (None when
        the writer is not native)."""
        if self._native is None or self.closed or not hasattr(self._native, "phase1_rows"):
            return None
        r = self.repos
        return (self._native, self.project_id, now, commit_hash, r.classes._INSERT, r.methods._INSERT)

    def put_project_update(self, project: Project) -> bool:
        """Queues ``project``'s row update (status, graph, commit hash) into the
        swap's transaction, so rows and project commit together (one commit
        instead of two, and no window where the new rows are visible under the
        old status).  True when queued; False when this writer cannot (Python
        writer, ``:memory:``): update the project after :meth:`wait` then."""
        if self._native is None or self.closed:
            return False
        for sql, params in self.repos.projects.update_statements(project):
            frozen = (params,)
            self._keep.append(frozen)
            self._native.put(sql, frozen)
        return True

    def close(self) -> None:
        """No more rows: the writer commits once everything queued is in."""
        self._closed = True
        if self._native is not None:
            self._native.commit()
        elif self._sync:
            self._write_all(iter(self._pending))
        else:
            self._q.put(None)

    def abort(self) -> None:
        self._done = True
        if self._native is not None:
            self._native.abort()
            self._keep.clear()
        elif self._thread is not None:
            self._q.put(("__abort__", ()))
            self._thread.join()

    def wait(self) -> int:
        if self._native is not None:
            if not self._done:
                self._done = True
                try:
                    self.rows_written = self._native.wait()
                    if hasattr(self._native, "timings"):
                        self.timings = self._native.timings()
                    self.repos.db.committed()
                except RuntimeError as e:
                    self._error = e
                self._keep.clear()
        elif self._thread is not None:
            self._thread.join()
        if self._error is not None:
            raise self._error
        return self.rows_written

    def __del__(self) -> None:
        # never release the row objects while the native thread may read them
        native = getattr(self, "_native", None)
        if native is not None and not getattr(self, "_done", True):
            try:
                if getattr(self, "_closed", False):
                    native.wait()
                else:
                    native.abort()  # never committed: roll back
            except Exception:
                pass

    # -------------------------------------------------------------- writer
    def _run(self) -> None:
        def batches():
            while True:
                item = self._q.get()
                if item is None:
                    return
                if item[0] == "__abort__":
                    raise _Aborted()
                yield item
        try:
            self._write_all(batches())
        except _Aborted:
            pass
        except BaseException as e:  # surfaced by wait()
            self._error = e
            while True:  # drain so a producer never blocks on us
                try:
                    if self._q.get_nowait() is None:
                        break
                except Exception:
                    break

    def _write_all(self, batches) -> None:
        r = self.repos
        with r.db.bulk_transaction():
            if self.replace:
                # children first: the FK cascade then finds nothing to do per row
                r.params.delete_by_project_id(self.project_id)
                r.methods.delete_by_project_id(self.project_id)
                r.classes.delete_by_project_id(self.project_id)
            for table, rows in batches:
                getattr(r, table).save_rows(rows)
                self.rows_written += len(rows)


class _Aborted(Exception):
    pass


def _native_bulk_writer():
    """``dmcp._srcscan.BulkWriter`` or None (module absent / predates it)."""
    try:
        from .. import _srcscan  # type: ignore
    except ImportError:
        return None
    return getattr(_srcscan, "BulkWriter", None)
