"""Indexing pipeline: analyze / re-analyze / rebuild / sync / resume
(CodeContextServiceTest, ProjectSyncServiceTest, AnalyzeProjectToolTest in the
reference) against real local git repositories and the offline fake backend."""
import json
import os
import subprocess
import threading

import pytest

from conftest import make_app
from dmcp.enrich.backend import FakeBackend, NullBackend
from dmcp.index.pipeline import common_package_prefix
from dmcp.models.domain import ProjectStatus
from dmcp.utils import synth
from dmcp.utils.errors import DomainError

O = "co.acme.shop.order"
U = "co.acme.shop.user"


def _git(root, *args):
    return subprocess.run(["git", "-C", str(root), *args], check=True, capture_output=True, text=True).stdout


@pytest.fixture
def repo(tmp_path):
    synth.java_spring_repo(str(tmp_path / "shop"), 16)
    return tmp_path / "shop"


def test_common_package_prefix():
    assert common_package_prefix(["co.a.b", "co.a.c", "co.a"]) == "co.a"
    assert common_package_prefix(["co.a.b", None, "org.x"]) == ""  # disjoint -> "" as in the reference
    assert common_package_prefix([]) is None and common_package_prefix([None]) is None
    assert common_package_prefix(["co.a.b"]) == "co.a.b"


def test_read_only_mode(tmp_path, repo):
    app = make_app(tmp_path, backend=NullBackend())
    with pytest.raises(DomainError) as e:
        app.indexer.analyze_project(str(repo))
    assert e.value.error_code == "READ_ONLY_MODE"
    assert app.repos.projects.find_all() == []
    app.close()


def test_analyze_persists_everything(tmp_path, repo):
    fake = FakeBackend()
    app = make_app(tmp_path, backend=fake)
    r = app.indexer.analyze_project(str(repo))
    assert r.success and r.classes_analyzed == 17 and r.endpoints_found == 10
    assert set(r.stats) >= {"analyze.clone", "analyze.parse", "analyze.phase1", "analyze.phase2", "classes"}
    p = app.repos.projects.find_by_id(r.project_id)
    assert p.status is ProjectStatus.ANALYZED and p.last_commit_hash == _git(repo, "rev-parse", "HEAD").strip()
    assert p.base_package == "co.acme.shop" and p.description.startswith("# shop")
    assert len(fake.calls) == 17 and app.repos.classes.find_unenriched_by_project_id(p.id) == []
    # the clone directory is cleaned up
    assert not any(os.scandir(tmp_path / "clones")) if (tmp_path / "clones").exists() else True
    # graph persisted == graph cached
    g = app.cache.get_graph(p.id)
    assert g.frozen and json.loads(p.graph_data)["nodes"].keys() == set(g.identifiers())
    assert g.node_info(f"{O}.OrderService").description.startswith("OrderService handles")
    app.close()


def test_reanalyze_is_idempotent_and_keeps_project(tmp_path, repo):
    app = make_app(tmp_path)
    r1 = app.indexer.analyze_project(str(repo))
    r2 = app.indexer.analyze_project(str(repo))
    assert r1.project_id == r2.project_id and r2.classes_analyzed == 17
    assert app.repos.classes.count_by_project()[r1.project_id] == 17
    n_params = app.db.query_one("SELECT COUNT(*) FROM method_parameters")[0]
    assert n_params > 0
    app.indexer.analyze_project(str(repo))
    assert app.db.query_one("SELECT COUNT(*) FROM method_parameters")[0] == n_params
    app.close()


def test_failed_enrichment_recovered_in_phase3(tmp_path, repo):
    seen = {}
    lock = threading.Lock()

    def flaky(inp):
        with lock:
            seen[inp.full_class_name] = seen.get(inp.full_class_name, 0) + 1
            first = seen[inp.full_class_name] == 1
        if first and inp.full_class_name.endswith("Service"):
            raise RuntimeError("rate limited")
        return json.dumps({"description": "ok " + inp.full_class_name, "classTypeCorrection": None, "methods": []})

    app = make_app(tmp_path, backend=FakeBackend(responder=flaky))
    r = app.indexer.analyze_project(str(repo))
    assert r.stats["enrichFailed"] == 2 and r.stats["recovered"] == 2
    assert app.repos.classes.find_unenriched_by_project_id(r.project_id) == []
    app.close()


def test_no_fix_missed_leaves_gaps_then_resume(tmp_path, repo):
    def broken(inp):
        if inp.full_class_name.endswith("Controller"):
            return "this is not json"
        return json.dumps({"description": "d", "methods": []})

    app = make_app(tmp_path, backend=FakeBackend(responder=broken))
    r = app.indexer.analyze_project(str(repo), fix_missed=False)
    missing = app.repos.classes.find_unenriched_by_project_id(r.project_id)
    assert {c.simple_name for c in missing} == {"OrderController", "UserController"}
    app.close()
    app2 = make_app(tmp_path)  # a later process with a working backend resumes
    out = app2.indexer.resume_enrichment(r.project_id)
    assert out == {"success": True, "projectId": r.project_id, "recovered": 2}
    assert app2.repos.classes.find_unenriched_by_project_id(r.project_id) == []
    g = app2.cache.get_graph(r.project_id)
    assert g.node_info(f"{O}.OrderController").description
    with pytest.raises(DomainError):
        app2.indexer.resume_enrichment("nope")
    app2.close()


def test_class_type_correction(tmp_path, repo):
    def corr(inp):
        c = {"OrderConfig": "SERVICE", "UserConfig": "NOT_A_TYPE", "Order": "null"}.get(
            inp.full_class_name.rsplit(".", 1)[-1])
        return json.dumps({"description": "x", "classTypeCorrection": c, "methods": []})

    app = make_app(tmp_path, backend=FakeBackend(responder=corr))
    app.indexer.analyze_project(str(repo))
    by = {c.simple_name: c.class_type.value for c in app.repos.classes.find_by_project_id(
        app.repos.projects.find_by_name("shop").id)}
    assert by["OrderConfig"] == "SERVICE" and by["UserConfig"] == "CONFIGURATION" and by["Order"] == "ENTITY"
    g = app.cache.get_graph_by_project_name("shop")
    assert g.node_info(f"{O}.OrderConfig").class_type == "SERVICE"
    app.close()


def test_static_only_analysis_when_allowed(tmp_path, repo):
    app = make_app(tmp_path, backend=NullBackend(), require_enrichment_for_analyze=False)
    r = app.indexer.analyze_project(str(repo))
    assert r.success and len(app.repos.classes.find_unenriched_by_project_id(r.project_id)) == 17
    app.close()


def test_rebuild_graph_keeps_enrichment(tmp_path, repo):
    app = make_app(tmp_path)
    r = app.indexer.analyze_project(str(repo))
    before = app.cache.get_graph(r.project_id)
    out = app.indexer.rebuild_graph(r.project_id)
    assert out["success"] and out["bound"] == 17 and out["parameters"] > 0
    after = app.cache.get_graph(r.project_id)
    assert after is not before
    assert after.node_info(f"{O}.OrderService").description == before.node_info(f"{O}.OrderService").description
    assert after.methods(f"{O}.OrderController") == before.methods(f"{O}.OrderController")
    assert after.method_parameters(f"{O}.OrderController") == before.method_parameters(f"{O}.OrderController")
    with pytest.raises(DomainError) as e:
        app.indexer.rebuild_graph("missing")
    assert e.value.error_code == "PROJECT_NOT_FOUND"
    app.close()


def test_sync_add_modify_delete(tmp_path, repo):
    fake = FakeBackend()
    app = make_app(tmp_path, backend=fake)
    r = app.indexer.analyze_project(str(repo))
    p = app.repos.projects.find_by_id(r.project_id)
    assert app.indexer.sync_project(p).to_dict()["addedClasses"] == 0  # no changes
    base = repo / "src/main/java/co/acme/shop"
    (base / "order/OrderConfig.java").unlink()
    svc = base / "user/UserService.java"
    svc.write_text(svc.read_text().replace("public class UserService {",
                                           "public class UserService {\n    public void audit() {}\n"))
    (base / "order/OrderAudit.java").write_text(
        "package co.acme.shop.order;\n\nimport co.acme.shop.user.UserService;\n\n"
        "@org.springframework.stereotype.Service\npublic class OrderAudit {\n"
        "    public void record(OrderRequest r) {}\n}\n")
    _git(repo, "add", "-A")
    _git(repo, "-c", "user.email=a@b", "-c", "user.name=t", "commit", "-qm", "change")
    fake.calls.clear()
    p = app.repos.projects.find_by_id(r.project_id)
    s = app.indexer.sync_project(p)
    assert s.success, s.error_message
    assert (s.added_classes, s.updated_classes, s.deleted_classes, s.unchanged_classes) == (1, 1, 1, 15)
    assert sorted(fake.calls) == [f"{O}.OrderAudit", f"{U}.UserService"]
    p = app.repos.projects.find_by_id(r.project_id)
    assert p.status is ProjectStatus.ANALYZED and p.last_commit_hash == s.commit_hash
    g = app.cache.get_graph(p.id)
    assert g.contains(f"{O}.OrderAudit") and not g.contains(f"{O}.OrderConfig")
    assert f"{U}.UserService" in g.dependencies(f"{O}.OrderAudit")
    assert "audit" in [m.method_name for m in g.methods(f"{U}.UserService")]
    # unchanged classes keep their enrichment in the republished graph
    assert g.node_info(f"{O}.OrderService").description.startswith("OrderService handles")
    ctx = app.context.get_method_context(f"{O}.OrderAudit", "record")
    assert ctx["found"] and ctx["parameterTypes"][0]["typeName"] == f"{O}.OrderRequest"
    assert app.repos.classes.count_by_project()[p.id] == 17
    app.close()


def test_sync_full_resync_when_old_commit_missing(tmp_path, repo):
    app = make_app(tmp_path)
    r = app.indexer.analyze_project(str(repo))
    p = app.repos.projects.find_by_id(r.project_id)
    p.last_commit_hash = "0" * 40
    app.repos.projects.update(p)
    s = app.indexer.sync_project(app.repos.projects.find_by_id(r.project_id))
    assert s.success and s.updated_classes == 17 and s.added_classes == 0


def test_sync_all_and_failure(tmp_path, repo):
    app = make_app(tmp_path)
    app.indexer.analyze_project(str(repo))
    res = app.indexer.sync_all_projects()
    assert res.success and res.total_projects == 1 and res.success_count == 1
    # repository gone -> failure recorded, project marked ERROR, others unaffected
    import shutil
    shutil.rmtree(repo)
    res = app.indexer.sync_all_projects()
    assert not res.success and res.failure_count == 1 and res.results[0].error_message
    assert app.repos.projects.find_by_name("shop").status is ProjectStatus.ERROR
    app.close()


def test_project_busy(tmp_path, repo):
    gate = threading.Event()
    release = threading.Event()

    def slow(inp):
        gate.set()
        release.wait(10)
        return json.dumps({"description": "d", "methods": []})

    app = make_app(tmp_path, backend=FakeBackend(responder=slow))
    t = threading.Thread(target=app.indexer.analyze_project, args=(str(repo),))
    t.start()
    assert gate.wait(20)
    with pytest.raises(DomainError) as e:
        app.indexer.analyze_project(str(repo))
    assert e.value.error_code == "PROJECT_BUSY"
    release.set()
    t.join(60)
    app.close()


def test_failed_prepare_releases_the_project_lock(tmp_path, repo, monkeypatch):
    """A failure while registering the project (e.g. ``database is locked``)
    must not leave the repository lock held: the next analysis runs."""
    app = make_app(tmp_path)
    real = app.indexer._prepare_project
    calls = []

    def flaky(url, branch):
        calls.append(1)
        if len(calls) == 1:
            raise RuntimeError("database is locked")
        return real(url, branch)

    monkeypatch.setattr(app.indexer, "_prepare_project", flaky)
    with pytest.raises(RuntimeError):
        app.indexer.analyze_project(str(repo))
    r = app.indexer.analyze_project(str(repo))  # not PROJECT_BUSY
    assert r.success and r.classes_analyzed > 0
    app.close()


def test_stuck_project_recovered_on_start(tmp_path, repo):
    app = make_app(tmp_path)
    r = app.indexer.analyze_project(str(repo))
    p = app.repos.projects.find_by_id(r.project_id)
    p.start_sync()
    app.repos.projects.update_status(p)
    app.close()
    app2 = make_app(tmp_path)
    assert app2.repos.projects.find_by_id(r.project_id).status is ProjectStatus.ERROR
    assert app2.indexer.sync_project(app2.repos.projects.find_by_id(r.project_id)).success
    app2.close()


def test_analysis_failure_marks_error(tmp_path):
    app = make_app(tmp_path)
    with pytest.raises(DomainError) as e:
        app.indexer.analyze_project(str(tmp_path / "does-not-exist"))
    assert e.value.error_code == "ANALYSIS_FAILED"
    p = app.repos.projects.find_by_name("does-not-exist")
    assert p is not None and p.status is ProjectStatus.ERROR
    app.close()


def test_nestjs_and_go_projects(tmp_path):
    synth.nestjs_repo(str(tmp_path / "nest"), 4)
    synth.go_gin_repo(str(tmp_path / "gosvc"), 3)
    app = make_app(tmp_path)
    rn = app.indexer.analyze_project(str(tmp_path / "nest"))
    rg = app.indexer.analyze_project(str(tmp_path / "gosvc"))
    assert rn.success and rn.classes_analyzed > 4 and rn.endpoints_found > 0
    assert rg.success and rg.classes_analyzed >= 3 and rg.endpoints_found > 0
    names = {p["name"] for p in app.context.list_projects()}
    assert names == {"nest", "gosvc"}
    api = app.context.get_service_api("gosvc")
    assert api["found"] and api["controllers"]
    app.close()


@pytest.mark.parametrize("stage", ["clone", "parse"])
def test_failed_reanalysis_keeps_previous_rows(tmp_path, repo, monkeypatch, stage):
    """The row swap's transaction opens before the snapshot is read (its
    deletes overlap clone + parse); a failure in either stage rolls it back,
    so the previous analysis survives (the reference deleted first,
    CodeContextService.java:745) and nothing waits on the open writer."""
    app = make_app(tmp_path)
    r = app.indexer.analyze_project(str(repo))
    n_methods = app.db.query_one("SELECT COUNT(*) FROM source_methods")[0]

    def boom(*a, **k):
        raise RuntimeError(f"{stage} failed")
    if stage == "clone":
        monkeypatch.setattr(app.indexer, "_fetch", boom)
    else:
        import dmcp.index.pipeline as pl
        monkeypatch.setattr(pl, "parser_for", boom)
    with pytest.raises(DomainError) as e:
        app.indexer.analyze_project(str(repo))
    assert e.value.error_code == "ANALYSIS_FAILED"
    assert app.repos.classes.count_by_project()[r.project_id] == 17
    assert app.db.query_one("SELECT COUNT(*) FROM source_methods")[0] == n_methods
    assert app.repos.projects.find_by_id(r.project_id).status is ProjectStatus.ERROR
    monkeypatch.undo()
    assert app.indexer.analyze_project(str(repo)).success  # lock released, writable again
    app.close()


def test_background_wal_checkpoints(tmp_path, repo):
    """Commits never checkpoint inline (wal_autocheckpoint = 0 on every
    connection, the native writer included); the database's checkpoint thread
    does, and the data is intact after a reopen."""
    app = make_app(tmp_path)
    r = app.indexer.analyze_project(str(repo))
    assert app.db.query_one("PRAGMA wal_autocheckpoint")[0] == 0
    ck = app.db.checkpointer
    assert ck is not None and ck._thread is not None
    app.close()
    assert ck.passes >= 1 and not ck._thread.is_alive()
    app2 = make_app(tmp_path)
    assert app2.repos.classes.count_by_project()[r.project_id] == 17
    assert app2.db.query_one("PRAGMA integrity_check")[0] == "ok"
    app2.close()
    app3 = make_app(tmp_path, db_background_checkpoint=False)
    assert app3.db.checkpointer is None and app3.db.query_one("PRAGMA wal_autocheckpoint")[0] == 1000
    app3.close()


def test_native_phase1_rows_match_python_loop(tmp_path, repo, monkeypatch):
    """Phase 1 built by the native writer (``phase1_rows``) writes the same
    rows -- ids included, given the same id sequence -- and the same graph
    metadata as the Python loop it replaces."""
    import dmcp.index.pipeline as pl
    from dmcp.index.pipeline import Indexer
    (repo / "src/main/java/co/acme/shop/order/Weird.java").write_text(
        "package co.acme.shop.order;\npublic class Weird {\n"
        "  public void boom() throws Erroré, java.io.IOException {}\n}\n")
    _git(repo, "add", "-A")
    _git(repo, "-c", "user.name=t", "-c", "user.email=t@t", "commit", "-qm", "weird")
    ids = [f"id-{i:06d}" for i in range(100000)]
    monkeypatch.setattr(pl, "new_ids", lambda n: ids[:n])
    monkeypatch.setattr(Indexer, "phase1_ids", ids)
    dumps = {}
    for native in (True, False):
        monkeypatch.setattr(Indexer, "native_phase1", native)
        app = make_app(tmp_path / f"n{int(native)}")
        r = app.indexer.analyze_project(str(repo))
        assert r.success
        tables = {t: app.db.query(f"SELECT * FROM {t} ORDER BY id") for t in
                  ("source_classes", "source_methods", "method_parameters")}
        rows = {t: [tuple(x[k] for k in x.keys() if k not in ("created_at", "project_id")) for x in v]
                for t, v in tables.items()}
        graph = json.loads(app.repos.projects.find_by_id(r.project_id).graph_data)
        dumps[native] = (rows, graph)
        app.close()
    assert dumps[True][0] == dumps[False][0]
    assert dumps[True][1] == dumps[False][1]
    exc = [x for x in dumps[True][0]["source_methods"] if x[2] == "boom"]
    assert exc and exc[0][5] == json.dumps(["Erroré", "java.io.IOException"])


def test_native_phase1_ids_are_time_ordered_uuid7(tmp_path, repo):
    """Without given ids the native Phase 1 mints UUIDv7s: unique, version 7,
    and increasing in row order (classes, then methods, appended to the
    primary-key B-trees)."""
    import re
    app = make_app(tmp_path)
    app.indexer.analyze_project(str(repo))
    g = app.cache.get_graph(app.repos.projects.find_all()[0].id)
    ids = [g.class_id(i) for i in g.identifiers()]  # minted in scan order, as the native scan writes them
    mids = [r[0] for r in app.db.query("SELECT id FROM source_methods")]
    pat = re.compile(r"^[0-9a-f]{8}-[0-9a-f]{4}-7[0-9a-f]{3}-[89ab][0-9a-f]{3}-[0-9a-f]{12}$")
    assert ids and all(pat.match(i) for i in ids + mids)
    assert len(set(ids + mids)) == len(ids) + len(mids)
    assert ids == sorted(ids)
    app.close()


@pytest.mark.parametrize("kind", ["java", "nest"])
def test_scan_written_rows_match_python_loop(tmp_path, monkeypatch, kind):
    """Class / method rows handed to the writer by the native scan itself
    (before the graph exists; Phase 1 then binds their ids and writes only the
    parameter rows) hold the same values, links and graph metadata as the
    Python Phase 1 loop -- compared by content, the ids being fresh UUIDv7s.
    Includes a non-ASCII exception name and an identifier defined twice
    (the later file wins)."""
    from dmcp.index.pipeline import Indexer
    repo = tmp_path / "src"
    if kind == "java":
        synth.java_spring_repo(str(repo), 24)
        (repo / "src/main/java/co/acme/shop/order/Weird.java").write_text(
            "package co.acme.shop.order;\npublic class Weird {\n"
            "  public void boom() throws Erroré, java.io.IOException, \\u0041x {}\n}\n")
    else:
        synth.nestjs_repo(str(repo), 4)
        (repo / "src" / "dup.ts").write_text("export function a(x: number) { return x; }\n")
        (repo / "src" / "dup.tsx").write_text("export function b() { return 1; }\n")
    _git(repo, "add", "-A")
    _git(repo, "-c", "user.name=t", "-c", "user.email=t@t", "commit", "-qm", "extra")

    def content(app, pid):
        cls = app.db.query("SELECT id, full_class_name, simple_name, package_name, class_type, description, "
                           "source_file, commit_hash FROM source_classes WHERE project_id = ?", (pid,))
        fq = {c["id"]: c["full_class_name"] for c in cls}
        meth = app.db.query("SELECT m.id, m.class_id, m.method_name, m.description, m.business_logic, "
                            "m.exceptions, m.http_method, m.http_path, m.line_number FROM source_methods m "
                            "JOIN source_classes c ON c.id = m.class_id WHERE c.project_id = ?", (pid,))
        mk = {m["id"]: (fq[m["class_id"]], m["method_name"], m["line_number"]) for m in meth}
        par = app.db.query("SELECT p.method_id, p.position, p.class_id FROM method_parameters p "
                           "JOIN source_methods m ON m.id = p.method_id JOIN source_classes c ON c.id = m.class_id "
                           "WHERE c.project_id = ?", (pid,))
        graph = json.loads(app.repos.projects.find_by_id(pid).graph_data)
        for node in graph["nodes"].values():
            node["classId"] = fq.get(node.get("classId"), node.get("classId"))
        return (sorted((tuple(c[k] for k in c.keys() if k != "id") for c in cls), key=repr),
                sorted(((fq[m["class_id"]],) + tuple(m[k] for k in m.keys() if k not in ("id", "class_id"))
                        for m in meth), key=repr),
                sorted(((mk[p["method_id"]], p["position"], fq[p["class_id"]]) for p in par), key=repr), graph)

    got = {}
    for native in (True, False):
        monkeypatch.setattr(Indexer, "native_phase1", native)
        app = make_app(tmp_path / f"n{int(native)}")
        r = app.indexer.analyze_project(str(repo))
        got[native] = content(app, r.project_id)
        if native:
            assert r.stats.get("analyze.writer_rows") is not None
        app.close()
    assert got[True][0] and got[True][1]
    assert got[True] == got[False]
    if kind == "java":
        assert any("\\u00e9" in (m[4] or "") for m in got[True][1])  # ensure_ascii form of the exception list


def test_slow_fetch_holds_no_database_write_lock(tmp_path):
    """The row swap's transaction (SQLite BEGIN IMMEDIATE: the database's
    write lock) is never held across a slow snapshot read: a local
    repository's swap opens early but is rolled back once the read outlasts
    ``early_swap_wait_s``, so while one analysis waits on a slow fetch another
    project's analysis and status writes go through, and the slow one still
    completes afterwards."""
    import time
    synth.java_spring_repo(str(tmp_path / "slow"), 6, base_package="co.slow", seed=3)
    synth.java_spring_repo(str(tmp_path / "fast"), 6, base_package="co.fast", seed=4)
    app = make_app(tmp_path)
    inside, release = threading.Event(), threading.Event()
    real = app.indexer._timed_fetch

    def fetch(url, branch):
        if url.value.endswith("slow"):
            inside.set()
            assert release.wait(60)
        return real(url, branch)
    app.indexer._timed_fetch = fetch
    out = {}
    t = threading.Thread(target=lambda: out.setdefault("slow", app.indexer.analyze_project(str(tmp_path / "slow"))))
    t.start()
    try:
        assert inside.wait(30)
        t0 = time.time()
        fast = app.indexer.analyze_project(str(tmp_path / "fast"))  # would wait the 30 s busy timeout
        assert fast.success and time.time() - t0 < 10
        assert app.repos.projects.find_by_id(fast.project_id).status == ProjectStatus.ANALYZED
    finally:
        release.set()
        t.join(60)
    assert out["slow"].success and out["slow"].classes_analyzed >= 6
    app.close()
