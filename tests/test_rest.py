"""REST API (AnalyzeProjectController / ProjectController / ContextController /
GraphQueryController / HealthController tests in the reference) and the CLI."""
import json

import pytest
from fastapi.testclient import TestClient

from conftest import make_app
from dmcp.__main__ import main as cli
from dmcp.api.rest import create_app
from dmcp.utils import synth

O = "co.acme.shop.order"


@pytest.fixture(scope="module")
def client(java_app):
    return TestClient(create_app(java_app))


def test_health_and_docs(client):
    r = client.get("/health")
    assert r.status_code == 200 and r.text == "up"
    spec = client.get("/api-docs").json()
    assert spec["info"]["title"] == "Domain MCP Server API"
    assert {"/api/projects/analyze", "/api/graph/query", "/api/context/stack-trace"} <= set(spec["paths"])
    assert client.get("/swagger-ui.html").status_code == 200


def test_projects_list_has_no_description(client):
    ps = client.get("/api/projects").json()["projects"]
    assert ps[0]["name"] == "shop" and "description" not in ps[0] and ps[0]["classCount"] == 17


def test_context_endpoints(client):
    assert client.get(f"/api/context/class/{O}.OrderService").json()["found"]
    assert client.get("/api/context/class", params={"className": f"{O}.OrderService"}).json()["found"]
    nf = client.get("/api/context/class", params={"className": "x.Y"})
    assert nf.status_code == 200 and nf.json()["found"] is False
    m = client.get("/api/context/method", params={"className": f"{O}.OrderController", "methodName": "list"})
    assert m.json()["httpEndpoint"] == "GET /"
    st = client.post("/api/context/stack-trace", json={"stackTrace": [
        {"className": f"{O}.OrderController", "methodName": "list", "lineNumber": 1}]}).json()
    assert st["executionPath"][0]["found"]


def test_graph_query_endpoint(client):
    r = client.post("/api/graph/query", json={"query": "shop:endpoints:+logic"})
    assert r.status_code == 200 and r.json()["count"] == 10
    bad = client.post("/api/graph/query", json={"query": "shop"})
    assert bad.status_code == 400 and bad.json()["errorCode"] == "INVALID_QUERY"
    missing = client.post("/api/graph/query", json={})
    assert missing.status_code == 400 and missing.json()["error"] == "Query is required"
    nf = client.post("/api/graph/query", json={"query": "ghost:endpoints"})
    assert nf.status_code == 400 and nf.json()["errorCode"] == "PROJECT_NOT_FOUND"


def test_tools_over_http_and_metrics(client):
    r = client.post("/api/tools/graph_query", json={"query": "shop:classes"}).json()
    assert not r["isError"] and json.loads(r["content"][0]["text"])["count"] == 17
    assert client.post("/api/tools/nope", json={}).status_code == 404
    text = client.get("/metrics").text
    assert "dmcp_" in text
    assert client.get("/api/stats").json()["graphsCached"] == 1


def test_analyze_rebuild_sync_over_http(tmp_path):
    synth.java_spring_repo(str(tmp_path / "inv"), 8)
    app = make_app(tmp_path)
    c = TestClient(create_app(app))
    r = c.post("/api/projects/analyze", json={"repositoryUrl": str(tmp_path / "inv")})
    body = r.json()
    assert r.status_code == 200 and body["success"] and body["classesAnalyzed"] == 9
    pid = body["projectId"]
    rb = c.post(f"/api/projects/{pid}/rebuild-graph").json()
    assert rb == {"success": True, "projectId": pid, "message": "Graph rebuilt successfully"}
    assert c.post("/api/projects/missing/rebuild-graph").status_code == 500
    s = c.post("/api/projects/sync").json()
    assert s["success"] and s["totalProjects"] == 1 and s["projects"][0]["projectName"] == "inv"
    assert c.post(f"/api/projects/{pid}/resume-enrichment").json()["recovered"] == 0
    bad = c.post("/api/projects/analyze", json={"repositoryUrl": "not a url"})
    assert bad.status_code == 500 and not bad.json()["success"]
    app.close()


def test_cli(tmp_path, capsys, monkeypatch):
    synth.java_spring_repo(str(tmp_path / "cli"), 8)
    db = str(tmp_path / "cli.db")
    monkeypatch.setenv("ENRICH_BACKEND", "fake")
    monkeypatch.setenv("GIT_CLONE_BASE_PATH", str(tmp_path / "clones"))
    assert cli(["--db", db, "analyze", str(tmp_path / "cli")]) == 0
    assert json.loads(capsys.readouterr().out)["classesAnalyzed"] == 9
    assert cli(["--db", db, "query", "cli:endpoints"]) == 0
    assert json.loads(capsys.readouterr().out)["count"] == 5
    assert cli(["--db", db, "tool", "search_project", '{"projectName": "cli", "query": "Order"}']) == 0
    assert json.loads(capsys.readouterr().out)["found"]
    assert cli(["--db", db, "query", "cli"]) == 2
    assert json.loads(capsys.readouterr().out)["errorCode"] == "INVALID_QUERY"
    assert cli(["--db", db, "list"]) == 0
    assert json.loads(capsys.readouterr().out)[0]["name"] == "cli"
    assert cli(["--db", db, "sync", "--project", "cli"]) == 0
    assert json.loads(capsys.readouterr().out)["success"]
    assert cli(["scan", str(tmp_path / "cli")]) == 0
    doc = json.loads(capsys.readouterr().out)
    assert doc["language"] == "java" and len(doc["files"]) == 9
