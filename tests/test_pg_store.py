"""PostgreSQL store: wire-protocol client (dmcp/store/pgwire.py), the
PgDatabase drop-in (dmcp/store/pg.py) and the whole service on it.

The reference persists to PostgreSQL (``application.yml:11-29``) and runs
its repository integration tests on Testcontainers ``postgres:14``.  No
PostgreSQL server or driver exists on this host, so these tests run the real
client against ``tests/pgfake.py`` -- a protocol-accurate server executing on
SQLite.  Protocol, authentication, pipelining, error and transaction
handling are pinned here; PostgreSQL-specific SQL semantics are parity
unpinned (no real server to compare with).
"""
import threading

import pytest

from dmcp.store.pg import PgDatabase, parse_postgres_url
from dmcp.store.pgwire import PgConnection, PgError, qmark_to_dollar
from tests.pgfake import FakePgServer


def _connect(srv, **kw):
    return PgConnection("127.0.0.1", srv.port, srv.user, kw.pop("password", srv.password), "testdb", **kw)


# ------------------------------------------------------------------ URLs
def test_parse_postgres_urls():
    t = parse_postgres_url("postgresql://bob:p%40ss@db.local:6543/index?currentSchema=domain_mcp&sslmode=disable")
    assert (t.host, t.port, t.user, t.password, t.database, t.schema, t.sslmode) == \
        ("db.local", 6543, "bob", "p@ss", "index", "domain_mcp", "disable")
    # the reference's JDBC form, credentials from DATABASE_USERNAME / _PASSWORD
    t = parse_postgres_url("jdbc:postgresql://localhost:5432/domain_mcp", "app", "pw")
    assert (t.user, t.password, t.port, t.schema) == ("app", "pw", 5432, None)
    # application.yml appends ?currentSchema=domain_mcp to a URL that already has it
    t = parse_postgres_url("jdbc:postgresql://h/db?currentSchema=domain_mcp?currentSchema=domain_mcp")
    assert t.schema == "domain_mcp" and t.database == "db"
    with pytest.raises(ValueError):
        parse_postgres_url("mysql://h/db")


def test_config_selects_postgres_from_env():
    from dmcp.config import Config
    cfg = Config.from_env({"DATABASE_URL": "jdbc:postgresql://h:5432/db?currentSchema=domain_mcp",
                           "DATABASE_USERNAME": "u", "DATABASE_PASSWORD": "p"})
    assert cfg.database_url.startswith("jdbc:postgresql://")
    assert (cfg.database_username, cfg.database_password) == ("u", "p")
    assert Config.from_env({"DATABASE_URL": "sqlite:////tmp/x.db"}).database_url is None


def test_qmark_translation_skips_literals():
    assert qmark_to_dollar("SELECT * FROM t WHERE a = ? AND b = '?' AND c IN (?, ?)") == \
        "SELECT * FROM t WHERE a = $1 AND b = '?' AND c IN ($2, $3)"


# ------------------------------------------------------------ authentication
@pytest.mark.parametrize("auth", ["trust", "password", "md5", "scram"])
def test_authentication_methods(tmp_path, auth):
    with FakePgServer(str(tmp_path / "a.sqlite"), auth=auth) as srv:
        c = _connect(srv)
        assert c.execute("SELECT 1 AS one").fetchone()["one"] == 1
        assert c.server_params["server_version"].startswith("14")
        c.close()
        if auth != "trust":
            with pytest.raises(PgError) as e:
                _connect(srv, password="wrong")
            assert e.value.sqlstate == "28P01"


# -------------------------------------------------------------- statements
def test_params_types_rowcounts_and_errors(pg_server):
    c = _connect(pg_server)
    c.execute_script("CREATE TABLE t (id VARCHAR(36) PRIMARY KEY, n INTEGER, note TEXT); "
                     "CREATE INDEX idx_t_n ON t(n)")
    assert c.execute("INSERT INTO t (id, n, note) VALUES (?, ?, ?)", ("a", 1, "héllo 'q' ?")).rowcount == 1
    assert c.execute("INSERT INTO t (id, n, note) VALUES ($1, $2, $3)", ("b", None, None)).rowcount == 1
    row = c.execute("SELECT id, n, note FROM t WHERE id = ?", ("a",)).fetchone()
    assert (row["id"], row[1], row["note"]) == ("a", 1, "héllo 'q' ?")
    assert c.execute("SELECT n FROM t WHERE id = ?", ("b",)).fetchone()[0] is None
    assert c.execute("UPDATE t SET n = ? WHERE n IS NULL", (7,)).rowcount == 1
    assert c.execute("DELETE FROM t WHERE id = ?", ("zzz",)).rowcount == 0
    with pytest.raises(PgError) as e:
        c.execute("INSERT INTO t (id, n) VALUES (?, ?)", ("a", 2))
    assert e.value.is_unique_violation
    assert c.tx_status == "I"  # autocommit: the session is usable again
    assert c.execute("SELECT COUNT(*) FROM t").fetchone()[0] == 2
    c.close()


def test_executemany_pipelines_chunks(pg_server):
    c = _connect(pg_server)
    c.PIPELINE_ROWS = 300  # several Sync-terminated chunks
    c.execute_script("CREATE TABLE r (id INTEGER PRIMARY KEY, v TEXT)")
    cur = c.executemany("INSERT INTO r (id, v) VALUES (?, ?)", ((i, f"v{i}") for i in range(1000)))
    assert cur.rowcount == 1000
    assert c.execute("SELECT COUNT(*), MAX(id) FROM r").fetchone()[:] == (1000, 999)
    # the INSERT was parsed once per connection and reused (prepared-statement cache)
    inserts = [s for s in pg_server.statements if s.startswith("INSERT INTO r")]
    assert len(inserts) == 1000
    c.close()


def test_transaction_failure_requires_rollback(pg_server):
    c = _connect(pg_server)
    c.execute_script("CREATE TABLE u (id INTEGER PRIMARY KEY)")
    c.execute("BEGIN")
    c.execute("INSERT INTO u (id) VALUES (?)", (1,))
    assert c.tx_status == "T"
    with pytest.raises(PgError):
        c.execute("INSERT INTO u (id) VALUES (?)", (1,))
    assert c.tx_status == "E"
    with pytest.raises(PgError) as e:  # PostgreSQL refuses everything until ROLLBACK
        c.execute("SELECT 1")
    assert e.value.sqlstate == "25P02"
    c.execute("ROLLBACK")
    assert c.tx_status == "I" and c.execute("SELECT COUNT(*) FROM u").fetchone()[0] == 0
    c.close()


def test_statement_cache_evicts_and_closes(pg_server):
    c = _connect(pg_server)
    c.STATEMENT_CACHE = 2
    for i in range(5):
        assert c.execute(f"SELECT {i} AS v WHERE 1 = ?", (1,)).fetchone()[0] == i
    assert len(c._stmts) == 2
    assert c.execute("SELECT 4 AS v WHERE 1 = ?", (1,)).fetchone()[0] == 4  # still cached
    c.close()


# ------------------------------------------------------------- PgDatabase
def test_pg_database_migrates_idempotently(pg_server):
    db = PgDatabase.from_url(pg_server.url())
    from dmcp.store.pg import PG_MIGRATIONS
    assert db.schema_version() == PG_MIGRATIONS[-1][0]
    assert db.migrate() == 0
    db2 = PgDatabase.from_url(pg_server.url())  # a second process adopts the schema
    assert db2.schema_version() == PG_MIGRATIONS[-1][0]
    db.close()
    db2.close()


def test_pg_repositories_and_row_writer(pg_server):
    from dmcp.models.domain import Project, RepositoryUrl
    from dmcp.store.repositories import Repositories
    db = PgDatabase.from_url(pg_server.url())
    repos = Repositories(db)
    p = Project.create("shop", RepositoryUrl.of("https://github.com/acme/shop.git"))
    repos.projects.save(p)
    for replace in (False, True):  # first analysis, then a re-analysis replacing the rows
        w = repos.project_rows_writer(p.id, replace=replace)
        assert w._native is None and w._thread is not None  # Python writer thread on PostgreSQL
        w.put("classes", [(f"c{replace}", p.id, "co.acme.Shop", "Shop", "co.acme", "SERVICE", None, "Shop.java",
                           "2026-10-16T00:00:00.000000Z", "abc")])
        w.put("methods", [(f"m{replace}", f"c{replace}", "buy", None, "[]", "[]", "POST", "/buy", 3,
                           "2026-10-16T00:00:00.000000Z")])
        w.put("params", [])
        w.close()
        w.wait()
    classes = repos.classes.find_by_project_id(p.id)
    assert [c.id for c in classes] == ["cTrue"]
    assert repos.methods.count_endpoints_by_project_id(p.id) == 1
    db.close()


def test_pg_threads_get_their_own_sessions(pg_server):
    db = PgDatabase.from_url(pg_server.url())
    seen = []

    def work():
        seen.append(id(db.conn.raw))
        db.query("SELECT 1")
    ts = [threading.Thread(target=work) for _ in range(3)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert len(set(seen)) == 3
    db.close()


def test_service_end_to_end_on_postgres(pg_server, tmp_path):
    """analyze -> persist -> MCP queries on the PostgreSQL store, then a fresh
    App (a restarted server) serves the graph loaded back from graph_data."""
    import json

    from dmcp.api.mcp_stdio import McpServer
    from dmcp.app import App
    from dmcp.config import Config
    from dmcp.enrich.backend import FakeBackend
    from dmcp.utils import synth
    fqcns = synth.java_spring_repo(str(tmp_path / "shop"), 12)
    cfg = Config(database_url=pg_server.url(), git_clone_base_path=str(tmp_path / "clones"),
                 recover_stuck_on_start=True)
    app = App(cfg, backend=FakeBackend())
    res = app.indexer.analyze_project(str(tmp_path / "shop"))
    assert res.success and res.classes_analyzed >= 12
    app.close()
    app2 = App(cfg, backend=FakeBackend())
    srv = McpServer(app2)

    def call(name, args):
        r = json.loads(srv.handle_line(json.dumps({"jsonrpc": "2.0", "id": 1, "method": "tools/call",
                                                   "params": {"name": name, "arguments": args}})))
        assert not r["result"]["isError"], r
        return json.loads(r["result"]["content"][0]["text"])
    projects = call("list_projects", {})
    assert projects[0]["name"] == "shop" and projects[0]["classCount"] == res.classes_analyzed
    q = call("graph_query", {"query": "shop:endpoints"})
    assert q["resultType"] == "endpoints" and q["count"] > 0
    svc = next(f for f in fqcns if f.endswith("OrderService"))
    ctx = call("get_class_context", {"className": svc, "projectName": "shop"})
    assert ctx["found"] and ctx["methods"] and ctx["description"]  # enrichment rows written through PostgreSQL
    method = ctx["methods"][0]["name"]
    trace = call("get_stack_trace_context", {"stackTrace": [{"className": svc, "methodName": method}]})
    assert trace["executionPath"][0]["found"]
    app2.close()


def test_pg_connections_only_set_the_search_path(pg_server):
    """A least-privilege role (USAGE/CREATE on the schema, no CREATE on the
    database) must be able to connect: only migrate() issues CREATE SCHEMA."""
    db = PgDatabase.from_url(pg_server.url())
    pg_server.statements.clear()
    db2 = PgDatabase.from_url(pg_server.url(), migrate=False)
    db2.query("SELECT COUNT(*) FROM projects")
    stmts = [s.upper() for s in pg_server.statements]
    assert not any("CREATE SCHEMA" in s for s in stmts)
    assert any(s.startswith("SET SEARCH_PATH") for s in stmts)
    db.close()
    db2.close()
