"""MCP stdio protocol + the nine tools (McpStdioServerConfigurationTest,
GraphQueryMcpToolTest and the *ToolTest classes in the reference)."""
import json
import os
import subprocess
import sys
import time

import pytest

from dmcp.api.mcp_stdio import McpServer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
O = "co.acme.shop.order"

TOOLS = {"list_projects", "get_class_context", "get_method_context", "get_stack_trace_context",
         "get_class_dependencies", "get_project_overview", "get_service_api", "search_project", "graph_query"}


def rpc(server, method, params=None, mid=1):
    msg = {"jsonrpc": "2.0", "id": mid, "method": method}
    if params is not None:
        msg["params"] = params
    return server.handle_message(msg)


def call(server, name, args):
    r = rpc(server, "tools/call", {"name": name, "arguments": args})["result"]
    assert r["content"][0]["type"] == "text" and len(r["content"]) == 1
    return r["isError"], (r["content"][0]["text"] if r["isError"] else json.loads(r["content"][0]["text"]))


def test_handshake_and_tools_list(java_app):
    s = McpServer(java_app)
    init = rpc(s, "initialize", {"protocolVersion": "2024-11-05", "capabilities": {},
                                 "clientInfo": {"name": "t", "version": "1"}})
    res = init["result"]
    assert res["protocolVersion"] == "2024-11-05" and res["serverInfo"] == {"name": "domain-mcp-server",
                                                                             "version": "1.0.1"}
    assert "tools" in res["capabilities"]
    assert rpc(s, "initialize", {"protocolVersion": "1999-01-01"})["result"]["protocolVersion"] == "2025-06-18"
    assert s.handle_message({"jsonrpc": "2.0", "method": "notifications/initialized"}) is None and s.initialized
    tools = rpc(s, "tools/list")["result"]["tools"]
    assert {t["name"] for t in tools} == TOOLS
    for t in tools:
        assert t["description"] and t["inputSchema"]["type"] == "object"
    gq = next(t for t in tools if t["name"] == "graph_query")
    assert gq["inputSchema"]["required"] == ["query"]
    assert rpc(s, "ping")["result"] == {}


def test_protocol_errors(java_app):
    s = McpServer(java_app)
    assert json.loads(s.handle_line("{not json"))["error"]["code"] == -32700
    assert s.handle_message({"id": 1, "method": "x"})["error"]["code"] == -32600
    assert rpc(s, "no/such")["error"]["code"] == -32601
    assert rpc(s, "tools/call", {"name": "nope"})["error"]["code"] == -32602
    assert rpc(s, "tools/call", {"arguments": {}})["error"]["code"] == -32602
    assert rpc(s, "tools/call", {"name": "list_projects", "arguments": [1]})["error"]["code"] == -32602
    assert s.handle_line("   ") is None
    batch = s.handle_message([{"jsonrpc": "2.0", "id": 1, "method": "ping"},
                              {"jsonrpc": "2.0", "method": "notifications/initialized"},
                              {"jsonrpc": "2.0", "id": 2, "method": "tools/list"}])
    assert [b["id"] for b in batch] == [1, 2]
    assert s.handle_message([])["error"]["code"] == -32600
    assert rpc(s, "resources/list")["result"] == {"resources": []}


def test_all_tools(java_app):
    s = McpServer(java_app)
    err, lp = call(s, "list_projects", {})
    assert not err and lp[0]["name"] == "shop"
    err, cc = call(s, "get_class_context", {"className": f"{O}.OrderService"})
    assert not err and cc["found"]
    err, mc = call(s, "get_method_context", {"className": f"{O}.OrderController", "methodName": "list"})
    assert not err and mc["httpEndpoint"] == "GET /"
    err, st = call(s, "get_stack_trace_context", {"stackTrace": [
        {"className": f"{O}.OrderController", "methodName": "list", "lineNumber": 17},
        {"className": f"{O}.OrderService", "methodName": "list", "lineNumber": "x"}, "junk"]})
    assert not err and len(st["executionPath"]) == 2 and st["executionPath"][0]["found"]
    err, cd = call(s, "get_class_dependencies", {"className": f"{O}.OrderService", "projectName": "shop"})
    assert not err and cd["found"]
    err, ov = call(s, "get_project_overview", {"projectName": "shop"})
    assert not err and ov["totalClasses"] == 17
    err, api = call(s, "get_service_api", {"projectName": "shop"})
    assert not err and api["controllers"]
    err, sp = call(s, "search_project", {"projectName": "shop", "query": "User"})
    assert not err and sp["matches"]
    err, q = call(s, "graph_query", {"query": "shop:endpoints"})
    assert not err and q["count"] == 10


def test_tool_errors_are_results(java_app):
    s = McpServer(java_app)
    err, text = call(s, "graph_query", {"query": "shop"})
    assert err and text.startswith("Error: Query must have at least project:target")
    err, text = call(s, "graph_query", {"query": "ghost:endpoints"})
    assert err and "Project not found: ghost" in text
    err, text = call(s, "get_class_context", {})
    assert err and text == "Error: Missing required argument: className"
    err, text = call(s, "get_stack_trace_context", {"stackTrace": "nope"})
    assert err
    # not-found is NOT an error
    err, nf = call(s, "get_class_context", {"className": "x.Nope"})
    assert not err and nf["found"] is False and nf["knownProjects"]


def test_stdio_subprocess_end_to_end(java_app, tmp_path):
    """Real process over pipes: stdout must carry only JSON-RPC lines (5 s budget
    per reply, as GraphQueryMcpToolTest)."""
    env = dict(os.environ, DMCP_DB_PATH=java_app.config.db_path, LOG_LEVEL="INFO",
               GIT_CLONE_BASE_PATH=str(tmp_path / "clones"), PYTHONPATH=ROOT)
    env.pop("ANTHROPIC_API_KEY", None)
    p = subprocess.Popen([sys.executable, "-m", "dmcp", "serve-mcp"], cwd=ROOT, env=env, stdin=subprocess.PIPE,
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, bufsize=1)
    try:
        msgs = [
            {"jsonrpc": "2.0", "id": 1, "method": "initialize",
             "params": {"protocolVersion": "2025-03-26", "capabilities": {}, "clientInfo": {"name": "x"}}},
            {"jsonrpc": "2.0", "method": "notifications/initialized"},
            {"jsonrpc": "2.0", "id": 2, "method": "tools/list"},
            {"jsonrpc": "2.0", "id": 3, "method": "tools/call",
             "params": {"name": "graph_query", "arguments": {"query": "shop:OrderController:methods"}}},
        ]
        replies = []
        for m in msgs:
            p.stdin.write(json.dumps(m) + "\n")
            p.stdin.flush()
            if "id" in m:
                t0 = time.time()
                line = p.stdout.readline()
                assert time.time() - t0 < 60  # first reply includes interpreter start-up
                replies.append(json.loads(line))
        assert [r["id"] for r in replies] == [1, 2, 3]
        assert replies[0]["result"]["protocolVersion"] == "2025-03-26"
        assert len(replies[1]["result"]["tools"]) == 9
        body = json.loads(replies[2]["result"]["content"][0]["text"])
        assert body["resultType"] == "methods" and body["count"] == 6  # constructor + 5 handlers
        assert body["results"][0]["methodName"] == "OrderController"
        t0 = time.time()
        p.stdin.write(json.dumps({"jsonrpc": "2.0", "id": 4, "method": "ping"}) + "\n")
        p.stdin.flush()
        assert json.loads(p.stdout.readline())["id"] == 4 and time.time() - t0 < 5
    finally:
        p.stdin.close()
        rc = p.wait(timeout=30)
        err = p.stderr.read()
        p.stdout.close()
        p.stderr.close()
    assert rc == 0, err
    assert "MCP stdio server is running" in err
