"""MCP server over stdio: newline-delimited JSON-RPC 2.0.

Parity: ``config/McpStdioServerConfiguration.java`` -- ``McpServer.sync`` over
``StdioServerTransportProvider`` with ``serverInfo("domain-mcp-server",
"1.0.1")`` and the tools capability (``:214-244``); the handshake exercised by
``GraphQueryMcpToolTest.java:191-235`` (``initialize`` -> ``notifications/
initialized`` -> ``tools/list`` / ``tools/call``).  The MCP Java SDK is not
available here, so the protocol layer is hand-written:

* requests get exactly one response line; notifications get none;
* protocol version negotiation (echo a supported client version, else ours);
* ``ping``, ``tools/list``, ``tools/call``; JSON-RPC errors -32700 parse,
  -32600 invalid request, -32601 method not found, -32602 invalid params;
* batch arrays are answered with an array;
* stdout carries protocol bytes only -- all logging goes to stderr.

Run: ``python -m dmcp serve-mcp`` (the reference's ``mcp`` profile).
"""
from __future__ import annotations

import json
import logging
import sys
import threading
from typing import Any, Dict, IO, List, Optional

from .tools import ToolRegistry

LOG = logging.getLogger(__name__)

SUPPORTED_PROTOCOL_VERSIONS = ["2025-06-18", "2025-03-26", "2024-11-05"]

PARSE_ERROR = -32700
INVALID_REQUEST = -32600
METHOD_NOT_FOUND = -32601
INVALID_PARAMS = -32602
INTERNAL_ERROR = -32603


class McpServer:
    def __init__(self, app, name: Optional[str] = None, version: Optional[str] = None) -> None:
        self.app = app
        self.registry = ToolRegistry(app)
        cfg = getattr(app, "config", None)
        self.name = name or (cfg.mcp_server_name if cfg else "domain-mcp-server")
        self.version = version or (cfg.mcp_server_version if cfg else "1.0.1")
        self.initialized = False
        self.client_info: Dict[str, Any] = {}
        self.protocol_version = SUPPORTED_PROTOCOL_VERSIONS[-1]
        self._write_lock = threading.Lock()

    # ----------------------------------------------------------- dispatch
    def handle_message(self, msg: Any) -> Optional[Any]:
        """Handles one decoded JSON value; returns the response object or None."""
        if isinstance(msg, list):
            if not msg:
                return _error(None, INVALID_REQUEST, "Invalid Request: empty batch")
            out = [r for r in (self.handle_message(m) for m in msg) if r is not None]
            return out or None
        if not isinstance(msg, dict) or msg.get("jsonrpc") != "2.0":
            return _error(msg.get("id") if isinstance(msg, dict) else None, INVALID_REQUEST, "Invalid Request")
        method = msg.get("method")
        has_id = "id" in msg
        mid = msg.get("id")
        if method is None:
            # a response from the client (e.g. to a server request) -- nothing to do
            return None
        if not isinstance(method, str):
            return _error(mid, INVALID_REQUEST, "Invalid Request: method must be a string")
        params = msg.get("params") or {}
        if not has_id:  # notification
            self._notification(method, params)
            return None
        try:
            result = self._request(method, params)
        except _RpcError as e:
            return _error(mid, e.code, e.message)
        except Exception as e:  # pragma: no cover - defensive
            LOG.exception("Internal error handling %s", method)
            return _error(mid, INTERNAL_ERROR, f"Internal error: {e}")
        return {"jsonrpc": "2.0", "id": mid, "result": result}

    def _notification(self, method: str, params: Dict[str, Any]) -> None:
        if method == "notifications/initialized":
            self.initialized = True
            LOG.info("MCP client initialized: %s", self.client_info)
        elif method == "notifications/cancelled":
            LOG.info("Client cancelled request %s", params.get("requestId"))
        else:
            LOG.debug("Ignoring notification %s", method)

    def _request(self, method: str, params: Dict[str, Any]) -> Any:
        if method == "initialize":
            requested = params.get("protocolVersion")
            self.protocol_version = requested if requested in SUPPORTED_PROTOCOL_VERSIONS \
                else SUPPORTED_PROTOCOL_VERSIONS[0]
            self.client_info = params.get("clientInfo") or {}
            return {"protocolVersion": self.protocol_version,
                    "capabilities": {"tools": {"listChanged": False}, "logging": {}},
                    "serverInfo": {"name": self.name, "version": self.version},
                    "instructions": "Use list_projects first, then get_stack_trace_context for stack traces "
                                    "or graph_query for structural navigation."}
        if method == "ping":
            return {}
        if method == "tools/list":
            return {"tools": self.registry.list()}
        if method == "tools/call":
            name = params.get("name")
            if not isinstance(name, str):
                raise _RpcError(INVALID_PARAMS, "Invalid params: tool name is required")
            args = params.get("arguments")
            if args is not None and not isinstance(args, dict):
                raise _RpcError(INVALID_PARAMS, "Invalid params: arguments must be an object")
            try:
                return self.registry.call(name, args)
            except KeyError:
                raise _RpcError(INVALID_PARAMS, f"Unknown tool: {name}")
        if method in ("resources/list", "prompts/list"):
            return {method.split("/")[0]: []}
        if method == "logging/setLevel":
            level = str(params.get("level", "info")).upper()
            logging.getLogger().setLevel({"WARNING": "WARNING", "ERROR": "ERROR", "DEBUG": "DEBUG"}.get(level, "INFO"))
            return {}
        raise _RpcError(METHOD_NOT_FOUND, f"Method not found: {method}")

    def handle_line(self, line: str) -> Optional[str]:
        line = line.strip()
        if not line:
            return None
        try:
            msg = json.loads(line)
        except ValueError as e:
            return json.dumps(_error(None, PARSE_ERROR, f"Parse error: {e}"))
        resp = self.handle_message(msg)
        if resp is None:
            return None
        return json.dumps(resp, ensure_ascii=False, separators=(",", ":"), default=str)

    # -------------------------------------------------------------- serve
    def serve(self, stdin: Optional[IO[str]] = None, stdout: Optional[IO[str]] = None) -> None:
        src = stdin or sys.stdin
        dst = stdout or sys.stdout
        LOG.info("MCP stdio server is running with %d tools. Waiting for input...", len(self.registry.tools))
        for line in src:
            out = self.handle_line(line)
            if out is not None:
                with self._write_lock:
                    dst.write(out + "\n")
                    dst.flush()
        LOG.info("stdin closed; MCP server exiting")


class _RpcError(Exception):
    def __init__(self, code: int, message: str) -> None:
        super().__init__(message)
        self.code = code
        self.message = message


def _error(mid: Any, code: int, message: str) -> dict:
    return {"jsonrpc": "2.0", "id": mid, "error": {"code": code, "message": message}}


def main(argv: Optional[List[str]] = None) -> int:
    from ..app import App, configure_logging
    from ..config import Config
    cfg = Config.from_env()
    configure_logging(cfg.log_level)
    app = App(cfg)
    try:
        McpServer(app).serve()
    finally:
        app.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
