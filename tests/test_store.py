"""SQLite store: migrations, repositories (ProjectRepositoryIntegrationTest,
SourceClassRepositoryIntegrationTest, SourceMethodRepositoryIntegrationTest)
and the query-plan check that replaces IndexAnalysisTest (Testcontainers
Postgres + EXPLAIN there; EXPLAIN QUERY PLAN on SQLite here)."""
import json
import threading

import pytest

from dmcp.models.domain import (ClassType, MethodParameter, Project, ProjectStatus, RepositoryUrl, SourceClass,
                                SourceMethod, new_id)
from dmcp.store.db import MIGRATIONS, Database
from dmcp.store.repositories import (MethodParameterRepository, Repositories, SourceClassRepository,
                                     SourceMethodRepository, from_iso, to_iso)


@pytest.fixture
def repos(tmp_db):
    return Repositories(tmp_db)


def _project(name="shop"):
    return Project.create(name, RepositoryUrl.of(f"https://github.com/acme/{name}.git"))


def test_migrations_idempotent(tmp_path):
    db = Database(str(tmp_path / "m.db"))
    assert db.schema_version() == MIGRATIONS[-1][0]
    assert db.migrate() == 0  # nothing left to apply
    names = {r[0] for r in db.query("SELECT name FROM sqlite_master WHERE type = 'index'")}
    assert "idx_source_methods_http_endpoints" in names and "idx_source_methods_class" not in names
    db.close()
    db2 = Database(str(tmp_path / "m.db"))
    assert db2.schema_version() == MIGRATIONS[-1][0]
    db2.close()


def test_graph_in_its_own_table(tmp_path):
    """Migration 9: the graph JSON lives in project_graphs (a status write
    never rewrites it); graphs already in projects.graph_data move over, the
    repository reads and writes them there, and deleting the project deletes
    its graph."""
    path = str(tmp_path / "g.db")
    db = Database(path)
    repos = Repositories(db)
    p = _project()
    p.update_graph_data('{"nodes":{"a":1}}')
    repos.projects.save(p)
    assert db.query_one("SELECT graph_data FROM projects WHERE id = ?", (p.id,))[0] is None
    assert db.query_one("SELECT graph_data FROM project_graphs WHERE project_id = ?", (p.id,))[0] == p.graph_data
    p.start_analysis()
    repos.projects.update_status(p)
    assert repos.projects.find_by_id(p.id).graph_data == '{"nodes":{"a":1}}'
    assert set(repos.projects.graph_versions()) == {p.id}
    assert [x.id for x in repos.projects.find_all_with_graph()] == [p.id]
    assert repos.projects.find_by_statuses([ProjectStatus.ANALYZING])[0].graph_data == p.graph_data
    p.update_graph_data(None)
    repos.projects.update(p)  # a full update without a graph removes it
    assert repos.projects.find_by_id(p.id).graph_data is None and repos.projects.graph_versions() == {}
    # a database from before migration 9 (the graph in the projects row)
    with db.transaction() as c:
        c.execute("UPDATE projects SET graph_data = ? WHERE id = ?", ('{"old":true}', p.id))
        c.execute("DROP TABLE project_graphs")
        c.execute("DELETE FROM schema_version WHERE version = 9")
    db.close()
    db = Database(path)
    repos = Repositories(db)
    assert repos.projects.find_by_id(p.id).graph_data == '{"old":true}'
    assert db.query_one("SELECT graph_data FROM projects WHERE id = ?", (p.id,))[0] is None
    repos.projects.delete(p.id)
    assert db.query_one("SELECT COUNT(*) FROM project_graphs")[0] == 0
    db.close()


def test_project_repository_roundtrip(repos):
    p = _project()
    p.update_description("d")
    repos.projects.save(p)
    got = repos.projects.find_by_id(p.id)
    assert got.name == "shop" and got.status is ProjectStatus.PENDING and got.description == "d"
    assert repos.projects.find_by_repository_url(p.repository_url).id == p.id
    assert repos.projects.find_by_name("shop").id == p.id and repos.projects.exists_by_repository_url(p.repository_url)
    p.start_analysis()
    p.analysis_completed("abc")
    p.update_graph_data('{"nodes":{}}')
    p.base_package = "co.acme"
    repos.projects.update(p)
    got = repos.projects.find_by_id(p.id)
    assert got.status is ProjectStatus.ANALYZED and got.last_commit_hash == "abc" and got.base_package == "co.acme"
    assert got.graph_data == '{"nodes":{}}' and got.last_analyzed_at is not None
    light = repos.projects.find_all()
    assert light[0].graph_data is None  # list views never load the graph blob
    assert repos.projects.find_all(with_graph=True)[0].graph_data
    assert [x.id for x in repos.projects.find_by_status(ProjectStatus.ANALYZED)] == [p.id]
    assert repos.projects.find_by_statuses([ProjectStatus.ERROR]) == []
    with pytest.raises(Exception):
        repos.projects.save(_project())  # unique repository_url
    repos.projects.delete(p.id)
    assert repos.projects.find_by_id(p.id) is None


def test_class_method_param_repositories(repos):
    p = _project()
    repos.projects.save(p)
    a = SourceClass.create(p.id, "co.acme.a.OrderService", ClassType.SERVICE, None, "src/A.java", "c1")
    b = SourceClass.create(p.id, "co.acme.b.Order", ClassType.ENTITY, "an order", "src/B.java", "c1")
    repos.classes.save_all([a, b])
    assert repos.classes.find_by_full_class_name("co.acme.a.OrderService").id == a.id
    assert repos.classes.count_by_project_id(p.id) == 2 and repos.classes.count_by_project() == {p.id: 2}
    assert repos.classes.class_type_breakdown(p.id) == {"SERVICE": 1, "ENTITY": 1}
    assert sorted(repos.classes.package_names(p.id)) == ["co.acme.a", "co.acme.b"]
    assert [c.id for c in repos.classes.find_by_package_prefix("co.acme")] == [b.id, a.id] or \
        {c.id for c in repos.classes.find_by_package_prefix("co.acme")} == {a.id, b.id}
    assert [c.id for c in repos.classes.find_unenriched_by_project_id(p.id)] == [a.id]
    repos.classes.update_enrichment(a.id, ClassType.CONTROLLER, "now a controller")
    assert repos.classes.find_by_id(a.id).class_type is ClassType.CONTROLLER
    by = repos.classes.find_by_full_class_names(["co.acme.b.Order", "missing"], project_id=p.id)
    assert set(by) == {"co.acme.b.Order"}

    m1 = SourceMethod.create(a.id, "create", None, None, ["E"], "POST", "/orders", 10)
    m2 = SourceMethod.create(a.id, "helper", None, None, None, None, None, 20)
    m3 = SourceMethod.create(a.id, "ctor", None, None, None, None, None, None)
    repos.methods.save_all([m3, m2, m1])
    assert [m.method_name for m in repos.methods.find_by_class_id(a.id)] == ["create", "helper", "ctor"]
    assert repos.methods.count_endpoints_by_project_id(p.id) == 1
    assert [m.id for m in repos.methods.find_http_endpoints_by_project_id(p.id)] == [m1.id]
    repos.methods.update_enrichment_batch([("creates", ["validate", "persist"], m1.id)])
    got = repos.methods.find_by_class_id_and_method_name(a.id, "create")
    assert got.description == "creates" and list(got.business_logic) == ["validate", "persist"] and list(got.exceptions) == ["E"]
    assert repos.methods.find_by_class_name_and_method_name("co.acme.a.OrderService", "helper").id == m2.id
    grouped = repos.methods.find_by_class_ids([a.id, b.id])
    assert len(grouped[a.id]) == 3 and not grouped.get(b.id)

    mp = MethodParameter.create(m1.id, 0, b.id)
    repos.params.save_all([mp])
    assert [x.class_id for x in repos.params.find_by_method_id(m1.id)] == [b.id]
    with pytest.raises(Exception):
        repos.params.save_all([MethodParameter.create(m1.id, 0, b.id)])  # unique (method, position)
    repos.params.delete_by_class_ids([a.id])
    repos.methods.delete_by_class_ids([a.id])
    repos.classes.delete_by_ids([a.id])
    assert repos.classes.count_by_project_id(p.id) == 1 and repos.params.find_by_method_id(m1.id) == []


def test_bulk_replace_keeps_referential_integrity(tmp_path):
    from conftest import make_app
    from dmcp.utils import synth
    synth.java_spring_repo(str(tmp_path / "shop"), 16)
    app = make_app(tmp_path)
    for _ in range(2):  # second run replaces every row inside bulk_transaction
        r = app.indexer.analyze_project(str(tmp_path / "shop"))
    assert app.db.query("PRAGMA foreign_key_check") == []
    assert app.db.query_one("PRAGMA foreign_keys")[0] == 1  # enforcement restored
    n = app.db.query_one("SELECT COUNT(*) FROM method_parameters p JOIN source_methods m ON m.id = p.method_id "
                         "JOIN source_classes c ON c.id = p.class_id WHERE c.project_id = ?", (r.project_id,))[0]
    assert n == app.db.query_one("SELECT COUNT(*) FROM method_parameters")[0] > 0
    # the invariant MethodParameterRepository.DELETE_BY_PROJECT_ID relies on:
    # a link's owning method and its target class belong to the same project
    assert app.db.query_one(
        "SELECT COUNT(*) FROM method_parameters p JOIN source_methods m ON m.id = p.method_id "
        "JOIN source_classes owner ON owner.id = m.class_id JOIN source_classes t ON t.id = p.class_id "
        "WHERE owner.project_id <> t.project_id")[0] == 0
    app.close()


def test_parameter_delete_by_class_id_matches_reference(repos):
    """``deleteByClassId`` removes links whose parameter TYPE is the class
    (``MethodParameterRepository.java:127-133``); the owner-side variant
    removes the links of the class's own methods."""
    p = _project()
    repos.projects.save(p)
    owner = SourceClass.create(p.id, "co.a.OrderService", ClassType.SERVICE, None, None, None)
    dto = SourceClass.create(p.id, "co.a.OrderDto", ClassType.DTO, None, None, None)
    other = SourceClass.create(p.id, "co.a.User", ClassType.ENTITY, None, None, None)
    repos.classes.save_all([owner, dto, other])
    m = SourceMethod.create(owner.id, "create", None, None, None, None, None, 1)
    repos.methods.save(m)
    repos.params.save_all([MethodParameter.create(m.id, 0, dto.id), MethodParameter.create(m.id, 1, other.id)])
    repos.params.delete_by_class_id(dto.id)  # type side only
    assert [x.class_id for x in repos.params.find_by_method_id(m.id)] == [other.id]
    repos.params.delete_by_class_id(owner.id)  # owner is no parameter type: nothing removed
    assert len(repos.params.find_by_method_id(m.id)) == 1
    repos.params.delete_by_owner_class_id(owner.id)
    assert repos.params.find_by_method_id(m.id) == []


def test_parameter_link_across_projects_rejected(repos):
    """The project-scoped delete selects links by target class; a link from one
    project's method to another project's class is refused at write time."""
    from dmcp.utils.errors import DomainError
    a, b = _project("a"), _project("b")
    repos.projects.save(a)
    repos.projects.save(b)
    ca = SourceClass.create(a.id, "co.a.Svc", ClassType.SERVICE, None, None, None)
    cb = SourceClass.create(b.id, "co.b.Dto", ClassType.DTO, None, None, None)
    repos.classes.save_all([ca, cb])
    m = SourceMethod.create(ca.id, "run", None, None, None, None, None, 1)
    repos.methods.save(m)
    with pytest.raises(DomainError) as e:
        repos.params.save_all([MethodParameter.create(m.id, 0, cb.id)])
    assert e.value.error_code == "PARAMETER_CROSS_PROJECT"
    with pytest.raises(DomainError):
        repos.params.save(MethodParameter.create(m.id, 0, cb.id))
    assert repos.params.find_by_method_id(m.id) == []
    repos.params.save(MethodParameter.create(m.id, 0, ca.id))  # same project: fine
    repos.params.delete_by_project_id(a.id)
    assert repos.params.find_by_method_id(m.id) == []


def test_cascade_delete_project(repos):
    p = _project()
    repos.projects.save(p)
    c = SourceClass.create(p.id, "x.Y", ClassType.OTHER, None, None, None)
    repos.classes.save(c)
    repos.methods.save(SourceMethod.create(c.id, "m", None, None, None, None, None, 1))
    repos.projects.delete(p.id)
    assert repos.classes.find_by_id(c.id) is None
    assert repos.db.query_one("SELECT COUNT(*) FROM source_methods")[0] == 0


def test_duplicate_fqcn_across_projects_picks_most_recent(repos):
    old, new = _project("a"), _project("b")
    for p, h in ((old, "h1"), (new, "h2")):
        repos.projects.save(p)
        p.start_analysis()
        p.analysis_completed(h)
        repos.projects.update(p)
    repos.db.execute("UPDATE projects SET last_analyzed_at = ? WHERE id = ?", ("2020-01-01T00:00:00Z", old.id))
    for p in (old, new):
        repos.classes.save(SourceClass.create(p.id, "co.shared.Util", ClassType.OTHER, None, None, None))
    assert repos.classes.find_by_full_class_name("co.shared.Util").project_id == new.id
    assert len(repos.classes.find_all_by_full_class_name("co.shared.Util")) == 2


def test_transactions_rollback_and_threads(tmp_db):
    repos = Repositories(tmp_db)
    p = _project()
    repos.projects.save(p)
    with pytest.raises(RuntimeError):
        with tmp_db.transaction():
            repos.classes.save(SourceClass.create(p.id, "x.A", ClassType.OTHER, None, None, None))
            raise RuntimeError("boom")
    assert repos.classes.count_by_project_id(p.id) == 0
    errors = []

    def worker(k):
        try:
            for i in range(20):
                repos.classes.save(SourceClass.create(p.id, f"t{k}.C{i}", ClassType.OTHER, None, None, None))
        except Exception as e:  # pragma: no cover
            errors.append(e)

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors and repos.classes.count_by_project_id(p.id) == 80


def test_iso_roundtrip():
    from datetime import datetime, timezone
    now = datetime(2024, 5, 6, 7, 8, 9, 123000, tzinfo=timezone.utc)
    assert from_iso(to_iso(now)) == now and to_iso(None) is None and from_iso(None) is None


# ----------------------------------------------------------- query plans
def _seed(repos, n_projects=50, classes_per=17, methods_per=3):
    """IndexAnalysisTest's fixture shape: 50 projects / 850 classes / 2,550 methods."""
    cls_rows, meth_rows = [], []
    for i in range(n_projects):
        p = _project(f"svc{i}")
        repos.projects.save(p)
        for j in range(classes_per):
            cid = new_id()
            pkg = f"co.acme.svc{i}.d{j % 4}"
            cls_rows.append((cid, p.id, f"{pkg}.C{j}", f"C{j}", pkg, "SERVICE", None, "f", "2024-01-01T00:00:00Z",
                             None))
            for k in range(methods_per):
                http = ("GET", f"/c{j}/{k}") if k == 0 else (None, None)
                meth_rows.append((new_id(), cid, f"m{k}", None, "[]", "[]", http[0], http[1], k + 1,
                                  "2024-01-01T00:00:00Z"))
    repos.classes.save_rows(cls_rows)
    repos.methods.save_rows(meth_rows)
    repos.db.execute("ANALYZE")


def _plan(db, sql, params):
    return " | ".join(r[3] for r in db.query("EXPLAIN QUERY PLAN " + sql, params))


def test_query_plans_use_indexes(repos):
    _seed(repos)
    db = repos.db
    pid = repos.projects.find_by_name("svc7").id
    cid = repos.classes.find_by_project_id(pid)[0].id
    cases = {
        "classes by project": (SourceClassRepository.FIND_BY_PROJECT_ID, (pid,)),
        "class by fqcn": (SourceClassRepository.FIND_BY_FULL_CLASS_NAME, ("co.acme.svc7.d1.C1",)),
        "class by project+fqcn": (SourceClassRepository.FIND_BY_PROJECT_ID_AND_FULL_CLASS_NAME,
                                  (pid, "co.acme.svc7.d1.C1")),
        "classes by package prefix": (SourceClassRepository.FIND_BY_PACKAGE_PREFIX,
                                      ("co.acme.svc7", "co.acme.svc7.", "co.acme.svc7/")),
        "unenriched": (SourceClassRepository.FIND_UNENRICHED_BY_PROJECT_ID, (pid,)),
        "methods by class": (SourceMethodRepository.FIND_BY_CLASS_ID, (cid,)),
        "method by class+name": (SourceMethodRepository.FIND_BY_CLASS_ID_AND_METHOD_NAME, (cid, "m1")),
        "endpoints by project": (SourceMethodRepository.FIND_HTTP_ENDPOINTS_BY_PROJECT_ID, (pid,)),
        "endpoint count": (SourceMethodRepository.COUNT_ENDPOINTS_BY_PROJECT_ID, (pid,)),
    }
    for name, (sql, params) in cases.items():
        plan = _plan(db, sql, params)
        # every filtered table is reached by an index search, never a full scan
        assert "SCAN source_classes" not in plan.replace("SCAN source_classes USING", "SEARCH"), (name, plan)
        assert "SCAN source_methods" not in plan.replace("SCAN source_methods USING", "SEARCH"), (name, plan)
        assert "SEARCH" in plan, (name, plan)
    # the partial endpoint index serves the endpoint queries
    assert "idx_source_methods_http_endpoints" in _plan(db, *cases["endpoints by project"]) or \
        "idx_source_methods_class_name" in _plan(db, *cases["endpoints by project"])


@pytest.mark.parametrize("mode", ["native", "pythread"])
def test_project_rows_writer_commit_abort_and_failure(tmp_path, monkeypatch, mode):
    """The background row swap commits everything, rolls back on abort, and
    surfaces a constraint failure from wait() with nothing half-written."""
    import dmcp.store.repositories as R
    from dmcp.store.db import Database
    if mode == "native":
        assert R._native_bulk_writer() is not None, "native BulkWriter missing from dmcp._srcscan"
    else:
        monkeypatch.setattr(R, "_native_bulk_writer", lambda: None)
    db = Database(str(tmp_path / "w.db"))
    repos = R.Repositories(db)
    p = _project()
    repos.projects.save(p)
    now = "2026-01-01T00:00:00.000000Z"

    def rows(tag):
        cls = [(f"c{tag}{i}", p.id, f"a.b.C{tag}{i}", f"C{tag}{i}", "a.b", "SERVICE", None, "F.java", now, "h")
               for i in range(50)]
        meth = [(f"m{tag}{i}", f"c{tag}{i // 2}", "run", None, "[]", "[]", None, None, i, now) for i in range(100)]
        par = [(f"p{tag}{i}", f"m{tag}{i}", 0, f"c{tag}{(i + 1) % 50}", now) for i in range(100)]
        return cls, meth, par

    def swap(tag, replace=True):
        w = repos.project_rows_writer(p.id, replace)
        c, m, pr = rows(tag)
        w.put("classes", c)
        w.put("methods", m)
        w.put("params", pr)
        return w

    w = swap("a", replace=False)
    w.close()
    assert w.wait() == 250
    assert repos.classes.count_by_project_id(p.id) == 50

    w = swap("b")
    w.abort()  # rolled back: generation "a" intact
    assert {c.full_class_name for c in repos.classes.find_by_project_id(p.id)} == {f"a.b.Ca{i}" for i in range(50)}

    w = repos.project_rows_writer(p.id, True)
    c, m, pr = rows("c")
    w.put("classes", c + c[:1])  # duplicate primary key -> the whole swap fails
    w.put("methods", m)
    w.close()
    with pytest.raises(Exception):
        w.wait()
    assert repos.classes.count_by_project_id(p.id) == 50
    assert db.query_one("SELECT COUNT(*) FROM method_parameters")[0] == 100

    w = swap("d")
    w.close()
    w.wait()
    names = {c.full_class_name for c in repos.classes.find_by_project_id(p.id)}
    assert names == {f"a.b.Cd{i}" for i in range(50)}
    assert db.query_one("SELECT COUNT(*) FROM source_methods")[0] == 100
    assert db.query("PRAGMA foreign_key_check") == []
    db.close()


def test_v6_clustered_tables_migration_keeps_rows(tmp_path, monkeypatch):
    """A database created before V6 (rowid tables, 4 KiB pages) migrates to
    the WITHOUT ROWID row tables with every row, constraint and index kept
    and foreign keys still enforced; new files get 16 KiB pages."""
    import sqlite3
    import dmcp.store.db as dbm
    from dmcp.store.db import Database
    from dmcp.store.repositories import Repositories
    path = str(tmp_path / "old.db")
    monkeypatch.setattr(dbm, "MIGRATIONS", [m for m in dbm.MIGRATIONS if m[0] < 6])
    monkeypatch.setattr(dbm, "PAGE_SIZE", 4096)
    old = Database(path)
    repos = Repositories(old)
    _seed(repos)
    with old.transaction() as c:  # parameter links: method -> a class of the same project
        c.execute("INSERT INTO method_parameters (id, method_id, position, class_id) "
                  "SELECT 'p' || m.id, m.id, 0, c.id FROM source_methods m JOIN source_classes c ON c.id = m.class_id")
    counts = {t: old.query_one(f"SELECT COUNT(*) FROM {t}")[0]
              for t in ("source_classes", "source_methods", "method_parameters")}
    assert all(counts.values()) and old.schema_version() == 5
    before = old.query("SELECT * FROM source_methods ORDER BY id")
    old.close()
    monkeypatch.undo()
    db = Database(path)
    assert db.schema_version() == MIGRATIONS[-1][0]
    for t, n in counts.items():
        assert db.query_one(f"SELECT COUNT(*) FROM {t}")[0] == n
        assert "WITHOUT ROWID" in db.query_one("SELECT sql FROM sqlite_master WHERE name = ?", (t,))[0]
    assert [tuple(r) for r in db.query("SELECT * FROM source_methods ORDER BY id")] == [tuple(r) for r in before]
    assert db.query("PRAGMA foreign_key_check") == []
    assert {r[2] for r in db.query("PRAGMA foreign_key_list(method_parameters)")} == {"source_methods",
                                                                                      "source_classes"}
    # cascades still work on the rebuilt tables
    pid = db.query_one("SELECT project_id FROM source_classes LIMIT 1")[0]
    with db.transaction() as c:
        c.execute("DELETE FROM projects WHERE id = ?", (pid,))
    assert db.query_one("SELECT COUNT(*) FROM source_classes WHERE project_id = ?", (pid,))[0] == 0
    with pytest.raises(sqlite3.IntegrityError):
        with db.transaction() as c:
            c.execute("INSERT INTO source_methods (id, class_id, method_name) VALUES ('x', 'no-such-class', 'm')")
    assert db.query_one("PRAGMA page_size")[0] == 4096  # an existing file keeps its page size
    db.close()
    fresh = Database(str(tmp_path / "new.db"))
    assert fresh.query_one("PRAGMA page_size")[0] == 16384
    fresh.close()
