"""PostgreSQL store: the reference's own database, over :mod:`dmcp.store.pgwire`.

The reference keeps its index in PostgreSQL, schema ``domain_mcp``
(``application.yml:11-29`` appends ``?currentSchema=domain_mcp``; Flyway
``db/migration/V1..V8``).  :class:`PgDatabase` is a drop-in for
:class:`dmcp.store.db.Database` -- same ``transaction`` / ``query`` /
``migrate`` API, so every repository (their SQL is written with ``?``
placeholders and portable syntax) runs unchanged -- which lets a deployment
point dmcp at the database the reference service already filled: the tables,
columns and types below are the reference's final schema (SURVEY §2.6,
components #49-#53), created only when missing, plus dmcp's one additive
column ``projects.base_package``.  dmcp tracks its own migrations in
``dmcp_schema_version`` and never touches Flyway's history table.

Selected with ``DATABASE_URL`` = ``postgresql://user:pass@host:5432/db`` or
the reference's JDBC form ``jdbc:postgresql://host:5432/db?currentSchema=...``
(with ``DATABASE_USERNAME`` / ``DATABASE_PASSWORD``, ``application.yml:12-14``).

Divergences from the SQLite store: the Phase-1 row swap runs on a Python
writer thread (the native bulk writer is SQLite-only) with pipelined
``executemany`` batches; foreign keys stay enforced (PostgreSQL has no
per-session switch for them without superuser rights).
"""
from __future__ import annotations

import contextlib
import logging
import threading
from dataclasses import dataclass, field
from typing import Dict, Iterator, List, Optional
from urllib.parse import parse_qs, unquote, urlparse

from .pgwire import PgConnection, PgCursor, PgError, PgRow

LOG = logging.getLogger(__name__)


@dataclass
class PgTarget:
    host: str = "127.0.0.1"
    port: int = 5432
    database: str = "postgres"
    user: str = "postgres"
    password: Optional[str] = None
    schema: Optional[str] = None
    sslmode: str = "prefer"
    options: Dict[str, str] = field(default_factory=dict)

    def describe(self) -> str:
        return f"postgresql://{self.user}@{self.host}:{self.port}/{self.database}" + \
            (f"?currentSchema={self.schema}" if self.schema else "")


def parse_postgres_url(url: str, user: Optional[str] = None, password: Optional[str] = None) -> PgTarget:
    """``postgresql://u:p@h:port/db?currentSchema=s&sslmode=...`` or the JDBC
    form ``jdbc:postgresql://h:port/db?currentSchema=s`` (credentials from
    ``user`` / ``password``, i.e. DATABASE_USERNAME / DATABASE_PASSWORD).
    A repeated query string (the reference's application.yml appends
    ``?currentSchema=domain_mcp`` to a URL that may already carry one,
    SURVEY §2.10) is tolerated: the first value of each key wins."""
    if url.startswith("jdbc:"):
        url = url[len("jdbc:"):]
    u = urlparse(url)
    if u.scheme not in ("postgres", "postgresql"):
        raise ValueError(f"not a PostgreSQL URL: {url}")
    query = (u.query or "").replace("?", "&")
    q = {k: v[0] for k, v in parse_qs(query, keep_blank_values=True).items()}
    t = PgTarget(host=u.hostname or "127.0.0.1", port=u.port or 5432,
                 database=unquote(u.path.lstrip("/")) or "postgres",
                 user=unquote(u.username) if u.username else (user or q.get("user") or "postgres"),
                 password=unquote(u.password) if u.password is not None else (password or q.get("password")),
                 schema=q.get("currentSchema") or q.get("currentschema") or q.get("search_path"),
                 sslmode=q.get("sslmode", "prefer"))
    return t


# The final schema of the reference's Flyway V1..V8 (tables V2 dropped are
# not created), written for PostgreSQL; IF NOT EXISTS everywhere so an
# existing reference database is adopted as is.
PG_MIGRATIONS = [
    (1, "reference_schema", """
CREATE TABLE IF NOT EXISTS projects (
    id               VARCHAR(36) PRIMARY KEY,
    name             VARCHAR(255) NOT NULL,
    repository_url   VARCHAR(500) NOT NULL UNIQUE,
    clone_location   VARCHAR(500),
    default_branch   VARCHAR(100) DEFAULT 'main',
    status           VARCHAR(50) NOT NULL DEFAULT 'PENDING',
    last_analyzed_at TIMESTAMP,
    last_commit_hash VARCHAR(40),
    created_at       TIMESTAMP NOT NULL DEFAULT CURRENT_TIMESTAMP,
    updated_at       TIMESTAMP NOT NULL DEFAULT CURRENT_TIMESTAMP,
    description      TEXT,
    graph_data       JSONB
);
CREATE INDEX IF NOT EXISTS idx_projects_status ON projects(status);
CREATE INDEX IF NOT EXISTS idx_projects_name ON projects(name);
CREATE TABLE IF NOT EXISTS source_classes (
    id              VARCHAR(36) PRIMARY KEY,
    project_id      VARCHAR(36) NOT NULL REFERENCES projects(id) ON DELETE CASCADE,
    full_class_name VARCHAR(500) NOT NULL,
    simple_name     VARCHAR(255) NOT NULL,
    package_name    VARCHAR(500),
    class_type      VARCHAR(50) NOT NULL,
    description     TEXT,
    source_file     VARCHAR(1000),
    created_at      TIMESTAMP NOT NULL DEFAULT CURRENT_TIMESTAMP,
    commit_hash     VARCHAR(40),
    UNIQUE (project_id, full_class_name)
);
CREATE INDEX IF NOT EXISTS idx_source_classes_full_name ON source_classes(full_class_name);
CREATE INDEX IF NOT EXISTS idx_source_classes_package ON source_classes(package_name);
CREATE INDEX IF NOT EXISTS idx_source_classes_project_package ON source_classes(project_id, package_name);
CREATE TABLE IF NOT EXISTS source_methods (
    id             VARCHAR(36) PRIMARY KEY,
    class_id       VARCHAR(36) NOT NULL REFERENCES source_classes(id) ON DELETE CASCADE,
    method_name    VARCHAR(255) NOT NULL,
    description    TEXT,
    business_logic TEXT,
    exceptions     TEXT,
    http_method    VARCHAR(10),
    http_path      VARCHAR(500),
    line_number    INTEGER,
    created_at     TIMESTAMP NOT NULL DEFAULT CURRENT_TIMESTAMP
);
CREATE INDEX IF NOT EXISTS idx_source_methods_class_name ON source_methods(class_id, method_name);
CREATE INDEX IF NOT EXISTS idx_source_methods_http_endpoints ON source_methods(class_id, http_path, http_method)
    WHERE http_method IS NOT NULL AND http_path IS NOT NULL;
CREATE TABLE IF NOT EXISTS method_parameters (
    id         VARCHAR(36) PRIMARY KEY,
    method_id  VARCHAR(36) NOT NULL REFERENCES source_methods(id) ON DELETE CASCADE,
    position   INTEGER NOT NULL,
    class_id   VARCHAR(36) NOT NULL REFERENCES source_classes(id) ON DELETE CASCADE,
    created_at TIMESTAMP NOT NULL DEFAULT CURRENT_TIMESTAMP,
    UNIQUE (method_id, position)
);
CREATE INDEX IF NOT EXISTS idx_method_params_class ON method_parameters(class_id);
"""),
    (2, "project_base_package", """
ALTER TABLE projects ADD COLUMN IF NOT EXISTS base_package TEXT;
"""),
    (3, "project_lease_and_graph_version", """
ALTER TABLE projects ADD COLUMN IF NOT EXISTS lease_owner VARCHAR(200);
ALTER TABLE projects ADD COLUMN IF NOT EXISTS lease_until DOUBLE PRECISION;
ALTER TABLE projects ADD COLUMN IF NOT EXISTS graph_version INTEGER NOT NULL DEFAULT 0;
"""),
    (4, "project_leases_table", """
CREATE TABLE IF NOT EXISTS project_leases (
    project_id  VARCHAR(36) PRIMARY KEY REFERENCES projects(id) ON DELETE CASCADE,
    lease_owner VARCHAR(200) NOT NULL,
    lease_until DOUBLE PRECISION NOT NULL
);
"""),
    (5, "class_enrichment_source", """
ALTER TABLE source_classes ADD COLUMN IF NOT EXISTS enrichment_source VARCHAR(600);
"""),
]


class PgDatabase:
    """PostgreSQL counterpart of :class:`dmcp.store.db.Database` (one
    connection per thread, explicit re-entrant transactions, migrations)."""

    native_bulk = False  # the native bulk writer speaks SQLite only
    path: Optional[str] = None

    def __init__(self, target: PgTarget, migrate: bool = True) -> None:
        self.target = target
        self._local = threading.local()
        self._conns: List[PgConnection] = []
        self._conns_lock = threading.Lock()
        if migrate:
            self.migrate()

    @classmethod
    def from_url(cls, url: str, user: Optional[str] = None, password: Optional[str] = None,
                 migrate: bool = True) -> "PgDatabase":
        return cls(parse_postgres_url(url, user, password), migrate=migrate)

    def describe(self) -> str:
        return self.target.describe()

    # ---------------------------------------------------------- connections
    def _open(self) -> PgConnection:
        t = self.target
        c = PgConnection(t.host, t.port, t.user, t.password, t.database, sslmode=t.sslmode, options=t.options)
        if t.schema:
            # only the search path per connection: CREATE SCHEMA needs CREATE on
            # the database even when the schema exists, which a least-privilege
            # application role (the reference's Flyway-managed deployment) lacks;
            # the schema is created once, by migrate()
            c.execute_script(f"SET search_path TO {self._schema_ident()}")
        with self._conns_lock:
            self._conns.append(c)
        return c

    @property
    def conn(self) -> "_PgConnAdapter":
        a = getattr(self._local, "conn", None)
        if a is None:
            a = self._local.conn = _PgConnAdapter(self._open())
        return a

    def is_shared_memory(self) -> bool:
        return False

    def close(self) -> None:
        with self._conns_lock:
            conns, self._conns = self._conns, []
        for c in conns:
            c.close()
        self._local = threading.local()

    # --------------------------------------------------------- transactions
    @contextlib.contextmanager
    def transaction(self) -> Iterator["_PgConnAdapter"]:
        conn = self.conn
        depth = getattr(self._local, "tx_depth", 0)
        if depth == 0:
            conn.execute("BEGIN")
        self._local.tx_depth = depth + 1
        try:
            yield conn
        except BaseException:
            self._local.tx_depth = depth
            if depth == 0:
                conn.execute("ROLLBACK")
            raise
        else:
            self._local.tx_depth = depth
            if depth == 0:
                conn.execute("COMMIT")

    @contextlib.contextmanager
    def bulk_transaction(self) -> Iterator["_PgConnAdapter"]:
        with self.transaction() as c:
            yield c

    def execute(self, sql: str, params=()) -> PgCursor:
        return self.conn.execute(sql, params)

    def query(self, sql: str, params=()) -> List[PgRow]:
        return self.conn.execute(sql, params).fetchall()

    def query_one(self, sql: str, params=()):
        rows = self.query(sql, params)
        return rows[0] if rows else None

    # ------------------------------------------------------------ migration
    def _schema_ident(self) -> str:
        return '"' + (self.target.schema or "").replace('"', '""') + '"'

    def migrate(self) -> int:
        conn = self.conn
        if self.target.schema:
            try:
                conn.raw.execute_script(f"CREATE SCHEMA IF NOT EXISTS {self._schema_ident()}")
            except PgError as e:  # no CREATE privilege: the schema must already exist
                LOG.info("CREATE SCHEMA %s skipped: %s", self.target.schema, e)
        conn.execute("CREATE TABLE IF NOT EXISTS dmcp_schema_version (version INTEGER PRIMARY KEY, "
                     "description TEXT, installed_on TIMESTAMP DEFAULT CURRENT_TIMESTAMP)")
        done = {r[0] for r in conn.execute("SELECT version FROM dmcp_schema_version").fetchall()}
        applied = 0
        for version, desc, sql in PG_MIGRATIONS:
            if version in done:
                continue
            try:
                with self.transaction() as c:
                    c.raw.execute_script(sql)
                    c.execute("INSERT INTO dmcp_schema_version(version, description) VALUES (?, ?)",
                              (version, desc))
            except PgError as e:
                if e.is_unique_violation:  # another process applied it concurrently
                    continue
                raise
            applied += 1
            LOG.info("Applied PostgreSQL migration V%d__%s", version, desc)
        return applied

    def schema_version(self) -> int:
        row = self.query_one("SELECT MAX(version) AS v FROM dmcp_schema_version")
        return int(row["v"] or 0)


class _PgConnAdapter:
    """The slice of the ``sqlite3.Connection`` API the repositories use."""

    def __init__(self, raw: PgConnection) -> None:
        self.raw = raw

    def execute(self, sql: str, params=()) -> PgCursor:
        return self.raw.execute(sql, tuple(params))

    def executemany(self, sql: str, seq) -> PgCursor:
        return self.raw.executemany(sql, seq)
