"""One test per case of the reference's ``GraphQueryMcpToolTest`` (6 cases).

Mirrors ``src/test/java/co/fanki/domainmcp/config/GraphQueryMcpToolTest.java``:
a real MCP server over a pair of in-process pipes (``PipedInputStream`` /
``PipedOutputStream`` there, ``os.pipe`` here), a fake LLM client that does
the ``initialize`` (protocol 2024-11-05) -> ``notifications/initialized``
handshake, then ``tools/list`` / ``tools/call graph_query`` with a 5 s read
budget per reply (``:191-235``), over the seeded ``order-service`` graph
(``buildOrderServiceGraph``, ``:237-272``).
"""
import json
import os
import queue
import threading

import pytest

from conftest import make_app
from dmcp.api.mcp_stdio import McpServer
from dmcp.graph.project_graph import MethodInfo, ProjectGraph


def order_service_graph():
    g = ProjectGraph()
    g.add_node("co.fanki.OrderController", "src/OrderController.java")
    g.add_node("co.fanki.OrderService", "src/OrderService.java")
    g.add_node("co.fanki.OrderRepository", "src/OrderRepository.java")
    g.add_dependency("co.fanki.OrderController", "co.fanki.OrderService")
    g.add_dependency("co.fanki.OrderService", "co.fanki.OrderRepository")
    g.mark_as_entry_point("co.fanki.OrderController")
    g.set_node_info("co.fanki.OrderController", "CONTROLLER", "Handles order HTTP requests")
    g.set_node_info("co.fanki.OrderService", "SERVICE", "Order business logic")
    g.set_node_info("co.fanki.OrderRepository", "REPOSITORY", "Order data access")
    g.add_method_info("co.fanki.OrderController", MethodInfo(
        "createOrder", "Creates a new order", ("Validate input", "Delegate to service", "Return 201"),
        ("ValidationException",), "POST", "/api/orders", 30))
    g.add_method_info("co.fanki.OrderController", MethodInfo(
        "getOrder", "Retrieves an order by ID", ("Lookup order", "Return order data"), ("NotFoundException",),
        "GET", "/api/orders/{id}", 45))
    return g


class PipedClient:
    """The fake LLM client on the other end of the server's stdin/stdout."""

    def __init__(self, server):
        c2s_r, c2s_w = os.pipe()
        s2c_r, s2c_w = os.pipe()
        self.server_in = os.fdopen(c2s_r, "r", encoding="utf-8")
        self.server_out = os.fdopen(s2c_w, "w", encoding="utf-8")
        self.writer = os.fdopen(c2s_w, "w", encoding="utf-8")
        self.reader = os.fdopen(s2c_r, "r", encoding="utf-8")
        self.lines: "queue.Queue[str]" = queue.Queue()
        self.thread = threading.Thread(target=server.serve, args=(self.server_in, self.server_out), daemon=True)
        self.thread.start()
        threading.Thread(target=self._pump, daemon=True).start()

    def _pump(self):
        for line in self.reader:
            self.lines.put(line)

    def send(self, obj):
        self.writer.write(json.dumps(obj) + "\n")
        self.writer.flush()

    def read_json(self, timeout=5.0):
        line = self.lines.get(timeout=timeout)  # "Server did not respond within 5 seconds"
        return json.loads(line)

    def close(self):
        self.writer.close()  # EOF on the server's stdin ends serve()
        self.thread.join(timeout=5)
        for f in (self.server_in, self.server_out, self.reader):
            try:
                f.close()
            except OSError:
                pass


@pytest.fixture
def client(tmp_path):
    app = make_app(tmp_path)
    app.cache.put("order-service-id", "order-service", order_service_graph())
    c = PipedClient(McpServer(app))
    c.send({"jsonrpc": "2.0", "id": 1, "method": "initialize",
            "params": {"protocolVersion": "2024-11-05", "capabilities": {},
                       "clientInfo": {"name": "test-llm", "version": "1.0"}}})
    init = c.read_json()
    assert init["result"]["protocolVersion"] == "2024-11-05"
    c.send({"jsonrpc": "2.0", "method": "notifications/initialized", "params": {}})
    yield c
    c.close()
    app.close()


def call_tool(c, mid, query):
    c.send({"jsonrpc": "2.0", "id": mid, "method": "tools/call",
            "params": {"name": "graph_query", "arguments": {"query": query}}})
    resp = c.read_json()
    assert resp["id"] == mid
    return resp["result"]


def test_when_listing_tools_should_include_graph_query_tool(client):
    client.send({"jsonrpc": "2.0", "id": 10, "method": "tools/list", "params": {}})
    tools = client.read_json()["result"]["tools"]
    gq = [t for t in tools if t["name"] == "graph_query"]
    assert gq, "graph_query tool must be registered"
    assert gq[0]["description"] and gq[0]["inputSchema"]["properties"]["query"]["type"] == "string"


def test_when_calling_graph_query_given_endpoints_query_should_return_endpoints(client):
    r = call_tool(client, 20, "order-service:endpoints")
    text = r["content"][0]["text"]
    assert not r["isError"] and "POST" in text and "/api/orders" in text


def test_when_calling_graph_query_given_classes_query_should_return_all_classes(client):
    r = call_tool(client, 21, "order-service:classes")
    text = r["content"][0]["text"]
    assert not r["isError"] and "OrderController" in text and "OrderService" in text


def test_when_calling_graph_query_given_methods_navigation_should_return_methods(client):
    r = call_tool(client, 22, "order-service:OrderController:methods")
    text = r["content"][0]["text"]
    assert not r["isError"] and "createOrder" in text and "getOrder" in text


def test_when_calling_graph_query_given_existence_check_should_return_true(client):
    r = call_tool(client, 23, "order-service:OrderController:?createOrder")
    assert not r["isError"] and json.loads(r["content"][0]["text"])["results"][0]["exists"] is True


def test_when_calling_graph_query_given_unknown_project_should_return_error(client):
    r = call_tool(client, 30, "nonexistent-service:endpoints")
    assert r["isError"] is True and r["content"][0]["text"].startswith("Error: ")
