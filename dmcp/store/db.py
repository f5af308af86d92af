"""SQLite database: connection management and versioned schema migrations.

The reference persists to PostgreSQL through Flyway migrations V1..V8
(``src/main/resources/db/migration``).  This store reproduces the *final*
schema of those migrations (components #49-#53) on SQLite:

* ``projects``          -- V1:13-27 + V5 ``description`` + V6 ``graph_data`` (stored in
  ``project_graphs`` since dmcp migration 9: the column stays, NULL)
* ``source_classes``    -- V1:149-165 + V8 ``commit_hash``; UNIQUE(project_id, full_class_name)
* ``source_methods``    -- V1:168-184 minus V8's dropped ``dependencies``
* ``method_parameters`` -- V7:6-19
* every index of V1/V3/V4/V7 (SQLite partial index for the endpoint index).

Additions (documented divergences): ``projects.base_package`` is stored at
analysis time so ``list_projects`` no longer loads every class of every
project (``CodeContextService.java:1752-1773``), and an ``updated_at`` trigger
mirrors ``V1:187-199``.  The V1 tables that V2 dropped are never created.

Concurrency: one connection per thread (WAL mode, ``foreign_keys=ON``,
``busy_timeout``), and :meth:`Database.transaction` gives an explicit
transaction per pipeline phase (the reference's ``@Transactional`` on
self-invoked package-private methods never actually opened one).
"""
from __future__ import annotations

import contextlib
import logging
import os
import sqlite3
import threading
import time
from typing import Iterator, List, Tuple

LOG = logging.getLogger(__name__)

MIGRATIONS: List[Tuple[int, str, str]] = [
    (1, "initial_schema", """
CREATE TABLE IF NOT EXISTS projects (
    id               TEXT PRIMARY KEY,
    name             TEXT NOT NULL,
    repository_url   TEXT NOT NULL UNIQUE,
    clone_location   TEXT,
    default_branch   TEXT DEFAULT 'main',
    status           TEXT NOT NULL DEFAULT 'PENDING',
    last_analyzed_at TEXT,
    last_commit_hash TEXT,
    created_at       TEXT NOT NULL DEFAULT (strftime('%Y-%m-%dT%H:%M:%fZ','now')),
    updated_at       TEXT NOT NULL DEFAULT (strftime('%Y-%m-%dT%H:%M:%fZ','now')),
    description      TEXT,
    graph_data       TEXT
);
CREATE INDEX IF NOT EXISTS idx_projects_status ON projects(status);
CREATE INDEX IF NOT EXISTS idx_projects_name ON projects(name);

CREATE TABLE IF NOT EXISTS source_classes (
    id              TEXT PRIMARY KEY,
    project_id      TEXT NOT NULL REFERENCES projects(id) ON DELETE CASCADE,
    full_class_name TEXT NOT NULL,
    simple_name     TEXT NOT NULL,
    package_name    TEXT,
    class_type      TEXT NOT NULL,
    description     TEXT,
    source_file     TEXT,
    created_at      TEXT NOT NULL DEFAULT (strftime('%Y-%m-%dT%H:%M:%fZ','now')),
    commit_hash     TEXT,
    CONSTRAINT uq_source_classes_project_class UNIQUE(project_id, full_class_name)
);
CREATE INDEX IF NOT EXISTS idx_source_classes_full_name ON source_classes(full_class_name);
CREATE INDEX IF NOT EXISTS idx_source_classes_package ON source_classes(package_name);
CREATE INDEX IF NOT EXISTS idx_source_classes_simple_name ON source_classes(simple_name);
CREATE INDEX IF NOT EXISTS idx_source_classes_type ON source_classes(class_type);
CREATE INDEX IF NOT EXISTS idx_source_classes_project_package ON source_classes(project_id, package_name);

CREATE TABLE IF NOT EXISTS source_methods (
    id             TEXT PRIMARY KEY,
    class_id       TEXT NOT NULL REFERENCES source_classes(id) ON DELETE CASCADE,
    method_name    TEXT NOT NULL,
    description    TEXT,
    business_logic TEXT,
    exceptions     TEXT,
    http_method    TEXT,
    http_path      TEXT,
    line_number    INTEGER,
    created_at     TEXT NOT NULL DEFAULT (strftime('%Y-%m-%dT%H:%M:%fZ','now'))
);
CREATE INDEX IF NOT EXISTS idx_source_methods_class ON source_methods(class_id);
CREATE INDEX IF NOT EXISTS idx_source_methods_name ON source_methods(method_name);
CREATE INDEX IF NOT EXISTS idx_source_methods_http_path ON source_methods(http_path);
CREATE INDEX IF NOT EXISTS idx_source_methods_class_name ON source_methods(class_id, method_name);
CREATE INDEX IF NOT EXISTS idx_source_methods_line ON source_methods(line_number)
    WHERE line_number IS NOT NULL;
CREATE INDEX IF NOT EXISTS idx_source_methods_http_endpoints
    ON source_methods(class_id, http_path, http_method)
    WHERE http_method IS NOT NULL AND http_path IS NOT NULL;

CREATE TABLE IF NOT EXISTS method_parameters (
    id         TEXT PRIMARY KEY,
    method_id  TEXT NOT NULL REFERENCES source_methods(id) ON DELETE CASCADE,
    position   INTEGER NOT NULL,
    class_id   TEXT NOT NULL REFERENCES source_classes(id) ON DELETE CASCADE,
    created_at TEXT NOT NULL DEFAULT (strftime('%Y-%m-%dT%H:%M:%fZ','now')),
    CONSTRAINT uq_method_param_position UNIQUE(method_id, position)
);
CREATE INDEX IF NOT EXISTS idx_method_params_method ON method_parameters(method_id);
CREATE INDEX IF NOT EXISTS idx_method_params_class ON method_parameters(class_id);
"""),
    (2, "optimize_query_indexes", """
-- V4 equivalent: covering index for ORDER BY full_class_name per project;
-- SQLite LIKE-prefix uses the plain package index (no text_pattern_ops).
CREATE INDEX IF NOT EXISTS idx_source_classes_project_ordered
    ON source_classes(project_id, full_class_name);
DROP INDEX IF EXISTS idx_source_classes_project;
CREATE TRIGGER IF NOT EXISTS update_projects_updated_at
    AFTER UPDATE ON projects FOR EACH ROW
    WHEN NEW.updated_at = OLD.updated_at
BEGIN
    UPDATE projects SET updated_at = strftime('%Y-%m-%dT%H:%M:%fZ','now') WHERE id = NEW.id;
END;
"""),
    (3, "project_base_package", """
ALTER TABLE projects ADD COLUMN base_package TEXT;
"""),
    (4, "drop_redundant_indexes", """
-- Measured with EXPLAIN QUERY PLAN over every repository statement
-- (tests/test_store.py::test_query_plans_use_indexes): none of these is the
-- chosen plan for any query, while each one costs a B-tree insert per row on
-- the indexing hot path.
--   idx_source_methods_class        prefix of idx_source_methods_class_name
--   idx_source_methods_name         no statement filters on method_name alone
--   idx_source_methods_http_path    endpoint queries use the partial index
--   idx_source_methods_line         no statement filters on line_number
--   idx_source_classes_simple_name  no statement filters on simple_name
--   idx_source_classes_type         breakdown is per project (project_package)
--   idx_source_classes_project_ordered  duplicate of the UNIQUE(project_id,
--                                   full_class_name) autoindex on SQLite
DROP INDEX IF EXISTS idx_source_methods_class;
DROP INDEX IF EXISTS idx_source_methods_name;
DROP INDEX IF EXISTS idx_source_methods_http_path;
DROP INDEX IF EXISTS idx_source_methods_line;
DROP INDEX IF EXISTS idx_source_classes_simple_name;
DROP INDEX IF EXISTS idx_source_classes_type;
DROP INDEX IF EXISTS idx_source_classes_project_ordered;
"""),
    (5, "drop_redundant_param_index", """
-- idx_method_params_method(method_id) is a prefix of the
-- UNIQUE(method_id, position) autoindex, which every lookup and the FK probe
-- already use (EXPLAIN QUERY PLAN); it only cost an extra insert per row.
DROP INDEX IF EXISTS idx_method_params_method;
"""),
    (6, "clustered_row_tables", """
-- foreign_keys: off
-- The three row tables as WITHOUT ROWID tables clustered on their
-- (time-ordered UUIDv7) primary key: the rowid table plus its separate
-- primary-key index were two B-trees per row; the whole-project swap of an
-- analysis inserts and deletes ~13k rows through them (measured on the
-- MI355X host with 16 KiB pages: 62 -> 55 ms per 2,001-class analysis).
-- Same columns, constraints and secondary indexes; rows copied over.
CREATE TABLE sc_new (
    id              TEXT PRIMARY KEY,
    project_id      TEXT NOT NULL REFERENCES projects(id) ON DELETE CASCADE,
    full_class_name TEXT NOT NULL,
    simple_name     TEXT NOT NULL,
    package_name    TEXT,
    class_type      TEXT NOT NULL,
    description     TEXT,
    source_file     TEXT,
    created_at      TEXT NOT NULL DEFAULT (strftime('%Y-%m-%dT%H:%M:%fZ','now')),
    commit_hash     TEXT,
    CONSTRAINT uq_source_classes_project_class UNIQUE(project_id, full_class_name)
) WITHOUT ROWID;
CREATE TABLE sm_new (
    id             TEXT PRIMARY KEY,
    class_id       TEXT NOT NULL REFERENCES source_classes(id) ON DELETE CASCADE,
    method_name    TEXT NOT NULL,
    description    TEXT,
    business_logic TEXT,
    exceptions     TEXT,
    http_method    TEXT,
    http_path      TEXT,
    line_number    INTEGER,
    created_at     TEXT NOT NULL DEFAULT (strftime('%Y-%m-%dT%H:%M:%fZ','now'))
) WITHOUT ROWID;
CREATE TABLE mp_new (
    id         TEXT PRIMARY KEY,
    method_id  TEXT NOT NULL REFERENCES source_methods(id) ON DELETE CASCADE,
    position   INTEGER NOT NULL,
    class_id   TEXT NOT NULL REFERENCES source_classes(id) ON DELETE CASCADE,
    created_at TEXT NOT NULL DEFAULT (strftime('%Y-%m-%dT%H:%M:%fZ','now')),
    CONSTRAINT uq_method_param_position UNIQUE(method_id, position)
) WITHOUT ROWID;
INSERT INTO sc_new (id, project_id, full_class_name, simple_name, package_name, class_type, description,
                    source_file, created_at, commit_hash)
    SELECT id, project_id, full_class_name, simple_name, package_name, class_type, description, source_file,
           created_at, commit_hash FROM source_classes;
INSERT INTO sm_new (id, class_id, method_name, description, business_logic, exceptions, http_method, http_path,
                    line_number, created_at)
    SELECT id, class_id, method_name, description, business_logic, exceptions, http_method, http_path,
           line_number, created_at FROM source_methods;
INSERT INTO mp_new (id, method_id, position, class_id, created_at)
    SELECT id, method_id, position, class_id, created_at FROM method_parameters;
DROP TABLE method_parameters;
DROP TABLE source_methods;
DROP TABLE source_classes;
ALTER TABLE sc_new RENAME TO source_classes;
ALTER TABLE sm_new RENAME TO source_methods;
ALTER TABLE mp_new RENAME TO method_parameters;
CREATE INDEX idx_source_classes_full_name ON source_classes(full_class_name);
CREATE INDEX idx_source_classes_package ON source_classes(package_name);
CREATE INDEX idx_source_classes_project_package ON source_classes(project_id, package_name);
CREATE INDEX idx_source_methods_class_name ON source_methods(class_id, method_name);
CREATE INDEX idx_source_methods_http_endpoints
    ON source_methods(class_id, http_path, http_method)
    WHERE http_method IS NOT NULL AND http_path IS NOT NULL;
CREATE INDEX idx_method_params_class ON method_parameters(class_id);
"""),
    (7, "project_lease_and_graph_version", """
-- Cross-process project lease (analyze / sync / rebuild / resume take it with
-- a conditional UPDATE and heartbeat it; lease_until is epoch seconds) and a
-- graph version bumped by every full project update, which lets the graph
-- cache of another process (the MCP server) notice a re-analysis.
ALTER TABLE projects ADD COLUMN lease_owner TEXT;
ALTER TABLE projects ADD COLUMN lease_until REAL;
ALTER TABLE projects ADD COLUMN graph_version INTEGER NOT NULL DEFAULT 0;
"""),
    (8, "project_leases_table", """
-- The lease moves to its own table (V7's projects.lease_owner / lease_until
-- are no longer written): SQLite rewrites the whole projects row, with its
-- multi-megabyte graph_data JSON, on every UPDATE of any column.
CREATE TABLE project_leases (
    project_id  TEXT PRIMARY KEY REFERENCES projects(id) ON DELETE CASCADE,
    lease_owner TEXT NOT NULL,
    lease_until REAL NOT NULL
) WITHOUT ROWID;
"""),
    (9, "project_graph_table", """
-- The graph JSON moves out of the projects row into its own table (SQLite
-- only; PostgreSQL keeps the reference's projects.graph_data): SQLite
-- rewrites a whole row, overflow pages included, on any UPDATE, so the
-- status write at the start of every analysis rewrote the previous
-- analysis' ~1.3 MB graph (~2 ms of a ~36 ms analysis on the MI355X host).
-- projects.graph_data stays, always NULL.
CREATE TABLE project_graphs (
    project_id TEXT PRIMARY KEY REFERENCES projects(id) ON DELETE CASCADE,
    graph_data TEXT NOT NULL
);
INSERT INTO project_graphs (project_id, graph_data)
    SELECT id, graph_data FROM projects WHERE graph_data IS NOT NULL;
UPDATE projects SET graph_data = NULL WHERE graph_data IS NOT NULL;
"""),
    (10, "class_enrichment_source", """
-- Which backend wrote a class's enrichment (dmcp.enrich.backend source
-- tags): 'synthetic:...' marks placeholder descriptions -- a random-weight
-- local preset, the echo engine, the offline fake -- that Phase 3 and
-- resume-enrichment redo once a real backend (a checkpoint, the API) is
-- configured.  NULL: never enriched, or enriched before this migration.
ALTER TABLE source_classes ADD COLUMN enrichment_source TEXT;
"""),
]

# New database files use 16 KiB pages (SQLite's default is 4 KiB): fewer
# B-tree levels and page splits for the row swap, fewer overflow pages for
# the multi-megabyte graph_data JSON (measured 62 -> 59 ms per analysis).
PAGE_SIZE = 16384


class _Checkpointer:
    """WAL checkpoints on a background thread instead of the committing one.

    SQLite's automatic checkpoint runs inside the COMMIT that pushes the WAL
    past 1,000 pages: the whole-project row swap of an analysis (~13k rows,
    ~8 MB of WAL) then pays for copying every page back into the database
    file and an fsync before its commit returns (measured 11-16 ms of a
    3 ms commit).  Here every connection runs with ``wal_autocheckpoint = 0``
    and each commit only wakes this thread, which runs a PASSIVE checkpoint
    (never blocks readers or writers) on its own connection; commits that
    arrive while it runs coalesce into one more pass.  Durability is that of
    ``synchronous = NORMAL`` in WAL mode either way."""

    def __init__(self, path: str) -> None:
        self.path = path
        self.passes = 0
        self._ev = threading.Event()
        self._stop = False
        self._thread: "threading.Thread | None" = None
        self._lock = threading.Lock()

    def notify(self) -> None:
        if self._thread is None:
            with self._lock:
                if self._thread is None and not self._stop:
                    self._thread = threading.Thread(target=self._run, name="dmcp-wal-checkpoint", daemon=True)
                    self._thread.start()
        self._ev.set()

    def _run(self) -> None:
        conn = sqlite3.connect(self.path, isolation_level=None, check_same_thread=False, timeout=30.0)
        try:
            while True:
                self._ev.wait()
                self._ev.clear()
                try:
                    conn.execute("PRAGMA wal_checkpoint(PASSIVE)").fetchall()
                    self.passes += 1
                except sqlite3.Error as e:  # busy with another process's checkpoint: the next commit retries
                    LOG.debug("background WAL checkpoint skipped: %s", e)
                if self._stop:
                    return
        finally:
            conn.close()

    def close(self) -> None:
        self._stop = True
        t = self._thread
        if t is not None:
            self._ev.set()  # one last pass, then exit
            t.join(timeout=60)


class Database:
    """Thread-local SQLite connections over one database file (or ``:memory:``).

    ``background_checkpoint`` (file databases): WAL checkpoints run on a
    :class:`_Checkpointer` thread after each commit instead of inside it."""

    # project graphs live in project_graphs (migration 9), not projects.graph_data
    graph_table = True

    def __init__(self, path: str = ":memory:", background_checkpoint: bool = True) -> None:
        self.path = path
        self._local = threading.local()
        self._write_lock = threading.RLock()
        self._shared_memory_conn = None
        self.checkpointer = _Checkpointer(path) if background_checkpoint and path != ":memory:" else None
        if path == ":memory:":
            # A private in-memory DB must be shared across threads via one connection.
            self._shared_memory_conn = self._open()
        else:
            d = os.path.dirname(os.path.abspath(path))
            os.makedirs(d, exist_ok=True)
        self.migrate()

    # ---------------------------------------------------------- connections
    def _open(self) -> sqlite3.Connection:
        conn = sqlite3.connect(self.path, check_same_thread=False, isolation_level=None,
                               timeout=30.0)
        conn.row_factory = sqlite3.Row
        conn.execute("PRAGMA foreign_keys = ON")
        if self.path != ":memory:":
            conn.execute(f"PRAGMA page_size = {PAGE_SIZE}")  # takes effect on a new, empty file only
            # switching to WAL needs a moment of exclusive access; concurrent
            # openers (bulk workers) get SQLITE_BUSY without the busy handler
            for attempt in range(200):
                try:
                    conn.execute("PRAGMA journal_mode = WAL")
                    break
                except sqlite3.OperationalError as e:
                    if "locked" not in str(e) or attempt == 199:
                        raise
                    time.sleep(0.05)
            conn.execute("PRAGMA synchronous = NORMAL")
            if self.checkpointer is not None:
                conn.execute("PRAGMA wal_autocheckpoint = 0")
        conn.execute("PRAGMA temp_store = MEMORY")
        conn.execute("PRAGMA cache_size = -65536")
        return conn

    def is_shared_memory(self) -> bool:
        """A private ``:memory:`` database: one connection shared by all threads."""
        return self._shared_memory_conn is not None

    @property
    def conn(self) -> sqlite3.Connection:
        if self._shared_memory_conn is not None:
            return self._shared_memory_conn
        c = getattr(self._local, "conn", None)
        if c is None:
            c = self._open()
            self._local.conn = c
        return c

    def committed(self) -> None:
        """A write transaction was committed (here or by the native bulk writer)."""
        if self.checkpointer is not None:
            self.checkpointer.notify()

    def close(self) -> None:
        if self.checkpointer is not None:
            self.checkpointer.close()
        c = getattr(self._local, "conn", None)
        if c is not None:
            c.close()
            self._local.conn = None
        if self._shared_memory_conn is not None:
            self._shared_memory_conn.close()
            self._shared_memory_conn = None

    # --------------------------------------------------------- transactions
    @contextlib.contextmanager
    def transaction(self) -> Iterator[sqlite3.Connection]:
        """Explicit write transaction (re-entrant: nested calls join the outer one)."""
        with self._write_lock:
            conn = self.conn
            depth = getattr(self._local, "tx_depth", 0)
            if self._shared_memory_conn is not None:
                depth = getattr(self, "_mem_tx_depth", 0)
            if depth == 0:
                conn.execute("BEGIN IMMEDIATE")
            self._set_depth(depth + 1)
            try:
                yield conn
            except BaseException:
                self._set_depth(depth)
                if depth == 0:
                    conn.execute("ROLLBACK")
                raise
            else:
                self._set_depth(depth)
                if depth == 0:
                    conn.execute("COMMIT")
                    self.committed()

    @contextlib.contextmanager
    def bulk_transaction(self) -> Iterator[sqlite3.Connection]:
        """A write transaction with foreign-key enforcement suspended on this
        connection, for the whole-project replace of Phase 1 (children deleted
        before parents, parents inserted before children: integrity is kept by
        construction, and ``tests/test_store.py`` runs ``foreign_key_check``).
        Skipping the per-row parent/child probes makes the swap ~20 % cheaper.
        Falls back to a plain transaction inside an open one."""
        conn = self.conn
        if self._shared_memory_conn is not None or getattr(self._local, "tx_depth", 0):
            with self.transaction() as c:
                yield c
            return
        with self._write_lock:
            conn.execute("PRAGMA foreign_keys = OFF")
            try:
                with self.transaction() as c:
                    yield c
            finally:
                conn.execute("PRAGMA foreign_keys = ON")

    def _set_depth(self, d: int) -> None:
        if self._shared_memory_conn is not None:
            self._mem_tx_depth = d
        else:
            self._local.tx_depth = d

    def execute(self, sql: str, params=()) -> sqlite3.Cursor:
        if self._shared_memory_conn is not None:
            with self._write_lock:
                return self.conn.execute(sql, params)
        return self.conn.execute(sql, params)

    def query(self, sql: str, params=()) -> List[sqlite3.Row]:
        if self._shared_memory_conn is not None:
            with self._write_lock:
                return self.conn.execute(sql, params).fetchall()
        return self.conn.execute(sql, params).fetchall()

    def query_one(self, sql: str, params=()):
        rows = self.query(sql, params)
        return rows[0] if rows else None

    # ------------------------------------------------------------ migration
    def migrate(self) -> int:
        with self._write_lock:
            conn = self.conn
            conn.execute("CREATE TABLE IF NOT EXISTS schema_version ("
                         "version INTEGER PRIMARY KEY, description TEXT, "
                         "installed_on TEXT DEFAULT (strftime('%Y-%m-%dT%H:%M:%fZ','now')))")
            done = {r[0] for r in conn.execute("SELECT version FROM schema_version")}
            applied = 0
            for version, desc, sql in MIGRATIONS:
                if version in done:
                    continue
                # a table rebuild runs with foreign keys off (a DROP TABLE would
                # otherwise cascade into the copies) and checks them before commit
                fk_off = "-- foreign_keys: off" in sql
                if fk_off:
                    conn.execute("PRAGMA foreign_keys = OFF")
                try:
                    conn.execute("BEGIN IMMEDIATE")
                    # another process may have applied it while we waited for the lock
                    if conn.execute("SELECT 1 FROM schema_version WHERE version = ?", (version,)).fetchone():
                        conn.execute("COMMIT")
                        continue
                    try:
                        for stmt in _split_sql(sql):
                            conn.execute(stmt)
                        if fk_off and conn.execute("PRAGMA foreign_key_check").fetchone():
                            raise sqlite3.IntegrityError(f"migration V{version}: foreign key check failed")
                        conn.execute("INSERT INTO schema_version(version, description) VALUES (?, ?)",
                                     (version, desc))
                        conn.execute("COMMIT")
                    except BaseException:
                        conn.execute("ROLLBACK")
                        raise
                finally:
                    if fk_off:
                        conn.execute("PRAGMA foreign_keys = ON")
                applied += 1
                LOG.debug("Applied migration V%d__%s", version, desc)
            return applied

    def schema_version(self) -> int:
        row = self.query_one("SELECT MAX(version) AS v FROM schema_version")
        return int(row["v"] or 0)


def _split_sql(script: str) -> List[str]:
    """Splits a migration script into statements (trigger bodies kept whole)."""
    out, buf, in_trigger = [], [], False
    for line in script.splitlines():
        stripped = line.strip()
        if not stripped or stripped.startswith("--"):
            continue
        buf.append(line)
        upper = stripped.upper()
        if upper.startswith("CREATE TRIGGER"):
            in_trigger = True
        if in_trigger:
            if upper == "END;":
                out.append("\n".join(buf))
                buf, in_trigger = [], False
            continue
        if stripped.endswith(";"):
            out.append("\n".join(buf))
            buf = []
    if buf:
        out.append("\n".join(buf))
    return out
