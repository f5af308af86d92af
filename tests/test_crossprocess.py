"""Two processes on one SQLite file: the project lease and graph-cache freshness.

The reference's two deployment modes (analysis service + MCP server,
SURVEY §1) share one database.  These tests run a real second Python process:

* an analysis in another process holds the project's lease: a concurrent
  analyze / sync / rebuild / resume here gets ``PROJECT_BUSY`` (reference:
  ANALYZING -> ANALYZING is illegal, ``ProjectStateMachine.java:34-70``);
* a holder that died (lease expired, status left ANALYZING) is taken over;
* an MCP server process answers ``graph_query`` for a project analyzed by
  another process, without a restart (``GraphService.java:55-146`` loads once).
"""
import json
import os
import subprocess
import sys
import time

import pytest

from conftest import ROOT, make_app
from dmcp.index.lease import ProjectLease
from dmcp.models.domain import ProjectStatus
from dmcp.utils import synth
from dmcp.utils.errors import DomainError

SLOW_ANALYZE = r"""
import sys, time
sys.path.insert(0, {root!r})
from dmcp.app import App
from dmcp.config import Config
from dmcp.enrich.backend import FakeBackend
cfg = Config(db_path={db!r}, git_clone_base_path={clones!r}, recover_stuck_on_start=False, enrich_stream=False)
app = App(cfg, backend=FakeBackend(max_concurrent=1, latency_s=0.15))
r = app.indexer.analyze_project({repo!r})
print("DONE", r.classes_analyzed, flush=True)
app.close()
"""


def _wait_status(app, url, status, timeout=60.0):
    t0 = time.time()
    while time.time() - t0 < timeout:
        p = app.repos.projects.find_by_repository_url(url, with_graph=False)
        if p is not None and p.status == status:
            return p
        time.sleep(0.05)
    raise AssertionError(f"project never reached {status}")


def test_concurrent_analyze_in_another_process_is_busy(tmp_path):
    repo = str(tmp_path / "shop")
    synth.java_spring_repo(repo, n_classes=24)
    app = make_app(tmp_path)
    code = SLOW_ANALYZE.format(root=ROOT, db=app.config.db_path, clones=str(tmp_path / "c2"), repo=repo)
    child = subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        p = _wait_status(app, os.path.abspath(repo), ProjectStatus.ANALYZING)
        owner, until = app.repos.projects.lease_of(p.id)
        assert owner and str(child.pid) in owner and until > time.time()
        with pytest.raises(DomainError) as e:
            app.indexer.analyze_project(repo)
        assert e.value.error_code == "PROJECT_BUSY"
        with pytest.raises(DomainError) as e:
            app.indexer.rebuild_graph(p.id)
        assert e.value.error_code == "PROJECT_BUSY"
        with pytest.raises(DomainError) as e:
            app.indexer.resume_enrichment(p.id)
        assert e.value.error_code == "PROJECT_BUSY"
        r = app.indexer.sync_project(p)
        assert not r.success and "already being processed" in r.error_message
        # a start-up recovery in this process must not break the live analysis
        assert app.recover_stuck_projects() == 0
        out, err = child.communicate(timeout=120)
        assert child.returncode == 0, err
        assert out.startswith("DONE 2")
    finally:
        if child.poll() is None:
            child.kill()
            child.wait()
    p = app.repos.projects.find_by_repository_url(os.path.abspath(repo), with_graph=False)
    assert p.status == ProjectStatus.ANALYZED and app.repos.projects.lease_of(p.id) == (None, None)
    r = app.indexer.analyze_project(repo)  # free again
    assert r.success
    app.close()


def test_expired_lease_of_a_dead_process_is_taken_over(tmp_path):
    repo = str(tmp_path / "shop")
    synth.java_spring_repo(repo, n_classes=16)
    app = make_app(tmp_path)
    assert app.indexer.analyze_project(repo).success
    p = app.repos.projects.find_by_repository_url(os.path.abspath(repo), with_graph=False)
    # a crashed analysis: status ANALYZING, lease of a process that stopped heartbeating
    with app.db.transaction() as c:
        c.execute("UPDATE projects SET status = 'ANALYZING' WHERE id = ?", (p.id,))
        c.execute("INSERT INTO project_leases (project_id, lease_owner, lease_until) VALUES (?, 'host:1:dead', ?)",
                  (p.id, time.time() + 30))
    with pytest.raises(DomainError) as e:  # not expired yet: busy
        app.indexer.analyze_project(repo)
    assert e.value.error_code == "PROJECT_BUSY"
    with app.db.transaction() as c:
        c.execute("UPDATE project_leases SET lease_until = ? WHERE project_id = ?", (time.time() - 1, p.id))
    r = app.indexer.analyze_project(repo)
    assert r.success
    p = app.repos.projects.find_by_id(p.id)
    assert p.status == ProjectStatus.ANALYZED and app.repos.projects.lease_of(p.id) == (None, None)
    app.close()


def test_lease_heartbeat_keeps_a_long_operation_alive(tmp_path):
    app = make_app(tmp_path)
    repo = str(tmp_path / "shop")
    synth.java_spring_repo(repo, n_classes=8)
    assert app.indexer.analyze_project(repo).success
    p = app.repos.projects.find_by_repository_url(os.path.abspath(repo), with_graph=False)
    with ProjectLease(app.repos.projects, p.id, ttl_s=1.2) as lease:
        time.sleep(2.5)  # > ttl: only the heartbeat keeps it
        with pytest.raises(DomainError):
            ProjectLease(app.repos.projects, p.id, ttl_s=1.2).acquire()
        lease.check()
        assert not lease.lost
    assert app.repos.projects.lease_of(p.id) == (None, None)
    # a lease that another process stole is reported at the next check
    lease = ProjectLease(app.repos.projects, p.id, ttl_s=1.2).acquire()
    with app.db.transaction() as c:
        c.execute("UPDATE project_leases SET lease_owner = 'other', lease_until = ? WHERE project_id = ?",
                  (time.time() + 60, p.id))
    time.sleep(0.9)
    with pytest.raises(DomainError) as e:
        lease.check()
    assert e.value.error_code == "LEASE_LOST"
    lease.release()
    assert app.repos.projects.lease_of(p.id)[0] == "other"  # release never frees another owner's lease
    app.close()


def _rpc(proc, mid, method, params=None):
    msg = {"jsonrpc": "2.0", "id": mid, "method": method}
    if params is not None:
        msg["params"] = params
    proc.stdin.write(json.dumps(msg) + "\n")
    proc.stdin.flush()
    return json.loads(proc.stdout.readline())


def _graph_query(proc, mid, q):
    r = _rpc(proc, mid, "tools/call", {"name": "graph_query", "arguments": {"query": q}})
    return r["result"]["isError"], r["result"]["content"][0]["text"]


def test_mcp_process_sees_analyses_of_another_process(tmp_path):
    app = make_app(tmp_path)
    env = dict(os.environ, DMCP_DB_PATH=app.config.db_path, LOG_LEVEL="WARNING", PYTHONPATH=ROOT,
               GIT_CLONE_BASE_PATH=str(tmp_path / "clones-mcp"), GRAPH_REFRESH_SECONDS="0.2")
    env.pop("ANTHROPIC_API_KEY", None)
    mcp = subprocess.Popen([sys.executable, "-m", "dmcp", "serve-mcp"], cwd=ROOT, env=env, stdin=subprocess.PIPE,
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, bufsize=1)
    try:
        assert _rpc(mcp, 1, "initialize", {"protocolVersion": "2024-11-05", "capabilities": {},
                                           "clientInfo": {"name": "t"}})["id"] == 1
        err, text = _graph_query(mcp, 2, "shop:endpoints")
        assert err and "not found" in text.lower()
        repo = str(tmp_path / "shop")
        synth.java_spring_repo(repo, n_classes=24)
        assert app.indexer.analyze_project(repo).success  # in THIS process
        time.sleep(0.3)
        err, text = _graph_query(mcp, 3, "shop:endpoints")
        assert not err, text
        first = json.loads(text)["count"]
        assert first > 0
        # a re-analysis with new endpoints is picked up too (graph_version moved)
        synth.java_spring_repo(repo, n_classes=48, seed=7)  # commits the larger tree
        assert app.indexer.analyze_project(repo).success
        time.sleep(0.3)
        err, text = _graph_query(mcp, 4, "shop:endpoints")
        assert not err and json.loads(text)["count"] > first
        # a deleted project disappears
        pid = app.repos.projects.find_by_name("shop").id
        app.projects.delete_project(pid)
        time.sleep(0.3)
        err, text = _graph_query(mcp, 5, "shop:endpoints")
        assert err
    finally:
        mcp.stdin.close()
        mcp.wait(timeout=30)
        mcp.stdout.close()
        mcp.stderr.close()
    app.close()


def test_lease_lives_in_its_own_table(tmp_path):
    """Lease writes never rewrite the projects row (its graph JSON is megabytes);
    deleting the project drops its lease."""
    app = make_app(tmp_path)
    repo = str(tmp_path / "shop")
    synth.java_spring_repo(repo, n_classes=8)
    assert app.indexer.analyze_project(repo).success
    p = app.repos.projects.find_by_repository_url(os.path.abspath(repo), with_graph=False)
    before = app.db.query_one("SELECT updated_at, graph_version FROM projects WHERE id = ?", (p.id,))
    lease = ProjectLease(app.repos.projects, p.id, ttl_s=30).acquire()
    assert app.repos.projects.lease_of(p.id)[0] == lease.owner
    assert app.repos.projects.try_acquire_lease(p.id, lease.owner, 30, time.time())  # re-entrant for its owner
    assert not app.repos.projects.try_acquire_lease(p.id, "someone-else", 30, time.time())
    after = app.db.query_one("SELECT updated_at, graph_version FROM projects WHERE id = ?", (p.id,))
    assert tuple(before) == tuple(after)
    lease.release()
    assert app.repos.projects.lease_of(p.id) == (None, None)
    ProjectLease(app.repos.projects, p.id, ttl_s=30).acquire()  # left held, then the project goes
    with app.db.transaction() as c:
        c.execute("DELETE FROM projects WHERE id = ?", (p.id,))
    assert app.db.query_one("SELECT COUNT(*) AS n FROM project_leases")["n"] == 0
    app.close()


def _hold_write_lock(db_path, seconds, then=None):
    """Another connection holds SQLite's write lock for ``seconds`` (a row
    swap longer than the lease TTL), optionally running ``then`` in it."""
    import sqlite3
    import threading
    ready = threading.Event()

    def run():
        c = sqlite3.connect(db_path, isolation_level=None, timeout=30)
        c.execute("BEGIN IMMEDIATE")
        ready.set()
        time.sleep(seconds)
        if then is not None:
            then(c)
        c.execute("COMMIT")
        c.close()
    t = threading.Thread(target=run, daemon=True)
    t.start()
    ready.wait(10)
    return t


def test_lease_not_renewed_past_its_ttl_fails_the_check(tmp_path):
    """The heartbeat blocked behind a write transaction longer than the TTL:
    the holder can no longer prove it owns the project, so check() fails
    (LEASE_LOST) instead of writing on; once renewals resume it holds again."""
    app = make_app(tmp_path, project_lease_seconds=1.0)
    repo = str(tmp_path / "shop")
    synth.java_spring_repo(repo, n_classes=4)
    assert app.indexer.analyze_project(repo).success
    p = app.repos.projects.find_by_repository_url(os.path.abspath(repo), with_graph=False)
    lease = ProjectLease(app.repos.projects, p.id, ttl_s=1.0).acquire()
    t = _hold_write_lock(app.config.db_path, 2.0)
    time.sleep(1.5)
    assert lease.expired() and lease.is_lost()
    with pytest.raises(DomainError) as e:
        lease.check()
    assert e.value.error_code == "LEASE_LOST"
    t.join(10)
    time.sleep(1.0)  # the blocked renewal went through after the lock
    lease.check()
    lease.release()
    app.close()


def test_analysis_that_loses_its_lease_leaves_the_new_owners_status(tmp_path):
    """A row swap held open past the TTL lets another process take the
    project over: the analysis stops at its next lease check and does NOT
    mark the project ERROR -- the status belongs to the new owner."""
    from dmcp.enrich.backend import FakeBackend
    repo = str(tmp_path / "shop")
    synth.java_spring_repo(repo, n_classes=40)
    holder = {}

    def responder(inp):
        if not holder:  # first class: another process's long transaction, then its takeover
            def takeover(c):
                pid = c.execute("SELECT id FROM projects").fetchone()[0]
                c.execute("UPDATE project_leases SET lease_owner = 'host:2:other', lease_until = ? "
                          "WHERE project_id = ?", (time.time() + 60, pid))
                c.execute("UPDATE projects SET status = 'SYNCING' WHERE id = ?", (pid,))
            holder["t"] = _hold_write_lock(app.config.db_path, 1.6, takeover)
            holder["t"].join(10)
        return '{"description": "d", "classTypeCorrection": null, "methods": []}'
    app = make_app(tmp_path, backend=FakeBackend(max_concurrent=1, responder=responder), project_lease_seconds=1.0)
    with pytest.raises(DomainError) as e:
        app.indexer.analyze_project(repo)
    assert "LEASE_LOST" in str(e.value.message) or "lease" in str(e.value.message).lower()
    p = app.repos.projects.find_by_repository_url(os.path.abspath(repo), with_graph=False)
    assert p.status == ProjectStatus.SYNCING  # not ERROR: the other owner's
    assert app.repos.projects.lease_of(p.id)[0] == "host:2:other"
    app.close()
