"""dmcp.parallel: distributed context (gloo, 2 ranks), bulk indexing
(in-process and worker processes), plus ProjectService and project deletion.
(The one-process-per-GPU enrichment workers: tests/test_workers.py.)"""
import json
import os
import socket
import threading

import pytest
import torch.multiprocessing as mp

from conftest import make_app
from dmcp.parallel.bulk import BulkItem, bulk_analyze, parse_repo_list
from dmcp.parallel.dist import init_from_env
from dmcp.utils import synth
from dmcp.utils.errors import DomainError


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    ctx = init_from_env(use_cuda=False)
    try:
        mx = ctx.max(float(rank + 1), -float(rank))
        sm = ctx.sum(float(rank + 1))
        objs = ctx.gather_objects({"rank": rank})
        ctx.synchronize()
        q.put((rank, mx, sm, objs))
    finally:
        ctx.shutdown()


def test_dist_context_single_process():
    ctx = init_from_env(use_cuda=False)
    assert ctx.world == 1 and ctx.is_main and ctx.device == "cpu"
    assert ctx.max(3.0, 1.0) == [3.0, 1.0] and ctx.sum(2.0) == [2.0] and ctx.gather_objects(7) == [7]
    ctx.synchronize()
    ctx.shutdown()


@pytest.mark.timeout(300)
def test_dist_context_two_ranks_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for rank, mx, sm, objs in got:
        assert mx == [2.0, 0.0] and sm == [3.0] and objs == [{"rank": 0}, {"rank": 1}]


def test_parse_repo_list():
    items = parse_repo_list("# comment\n\nhttps://github.com/a/b.git develop\n/srv/repo\n")
    assert items == [BulkItem("https://github.com/a/b.git", "develop"), BulkItem("/srv/repo", None)]


def test_bulk_analyze_in_process_and_workers(tmp_path):
    for i in range(3):
        synth.java_spring_repo(str(tmp_path / f"r{i}"), 8, base_package=f"co.r{i}")
    items = [BulkItem(str(tmp_path / f"r{i}")) for i in range(3)] + [BulkItem(str(tmp_path / "missing"))]
    app = make_app(tmp_path, enrich_backend="fake")
    res = bulk_analyze(app.config, items[:2], workers=1, app=app)
    assert [r.success for r in res] == [True, True] and res[0].classes == 9
    app.close()
    from dmcp.config import Config
    cfg = Config(db_path=str(tmp_path / "bulk.db"), git_clone_base_path=str(tmp_path / "c2"),
                 enrich_backend="fake")
    res2 = bulk_analyze(cfg, items, workers=3)
    assert [r.success for r in res2] == [True, True, True, False]
    assert "Analysis failed" in res2[3].message
    app2 = make_app(tmp_path, db_path=str(tmp_path / "bulk.db"))
    assert {p["name"] for p in app2.context.list_projects()} == {"r0", "r1", "r2", "missing"}
    app2.close()


def test_project_service_and_delete(tmp_path):
    synth.java_spring_repo(str(tmp_path / "shop"), 8)
    app = make_app(tmp_path)
    svc = app.projects
    p = svc.register_project("x", "https://github.com/acme/x.git", "dev")
    assert p.default_branch == "dev" and svc.get_by_id(p.id).name == "x"
    with pytest.raises(DomainError) as e:
        svc.register_project("x2", "https://github.com/acme/x.git")
    assert e.value.error_code == "PROJECT_ALREADY_EXISTS"
    with pytest.raises(DomainError) as e:
        svc.get_by_id("nope")
    assert e.value.error_code == "PROJECT_NOT_FOUND"
    svc.mark_analysis_started(p.id)
    with pytest.raises(DomainError):
        svc.delete_project(p.id)  # busy
    svc.mark_analysis_completed(p.id, "abc")
    assert svc.find_by_repository_url("https://github.com/acme/x.git").last_commit_hash == "abc"
    from dmcp.models.domain import ProjectStatus
    assert [x.id for x in svc.list_by_status(ProjectStatus.ANALYZED)] == [p.id]
    assert len(svc.list_projects()) == 1
    r = app.indexer.analyze_project(str(tmp_path / "shop"))
    assert app.cache.get_graph(r.project_id) is not None
    assert svc.delete_project(r.project_id) and not svc.delete_project(r.project_id)
    assert app.cache.get_graph(r.project_id) is None and app.repos.classes.count_by_project_id(r.project_id) == 0
    assert app.graph_query.cache.get_graph_by_project_name("shop") is None
    app.close()


def test_cli_analyze_batch_and_delete(tmp_path, capsys, monkeypatch):
    from dmcp.__main__ import main as cli
    synth.java_spring_repo(str(tmp_path / "a"), 8)
    lst = tmp_path / "repos.txt"
    lst.write_text(f"# repos\n{tmp_path / 'a'}\n{tmp_path / 'nope'}\n")
    monkeypatch.setenv("ENRICH_BACKEND", "fake")
    monkeypatch.setenv("GIT_CLONE_BASE_PATH", str(tmp_path / "clones"))
    db = str(tmp_path / "cli.db")
    assert cli(["--db", db, "analyze-batch", str(lst)]) == 1  # one failure
    out = json.loads(capsys.readouterr().out)
    assert out["total"] == 2 and out["success"] == 1
    pid = out["results"][0]["project_id"]
    assert cli(["--db", db, "delete", pid]) == 0
    assert json.loads(capsys.readouterr().out)["success"]
    assert cli(["--db", db, "delete", pid]) == 1
