"""The nine MCP tools: names, descriptions, JSON schemas and handlers.

Parity: ``config/McpStdioServerConfiguration.java`` -- schemas ``:45-192``,
tool specs ``:259-552``, ``toCallToolResult`` (``:554-563``: the result
serialized as ONE text content item) and ``errorResult`` (``:565-570``:
``isError=true`` with ``"Error: <message>"``).  "Not found" is not an error:
those tools return ``found=false`` + ``knownProjects``.
"""
from __future__ import annotations

import json
import logging
from dataclasses import dataclass
from typing import Any, Callable, Dict, List, Optional

from ..utils.errors import DomainError
from ..utils.tracing import span

LOG = logging.getLogger(__name__)

_PROJECT_SCOPE = "Optional: scope the search to this project (as returned by list_projects)"
_CLASS_NAME = {"type": "string", "description": "The fully qualified class name"}
_PROJECT_NAME = {"type": "string", "description": "The project name as returned by list_projects"}


@dataclass
class Tool:
    name: str
    description: str
    input_schema: dict
    handler: Callable[[Dict[str, Any]], Any]

    def spec(self) -> dict:
        return {"name": self.name, "description": self.description, "inputSchema": self.input_schema}


class ToolError(Exception):
    pass


def _require(args: Dict[str, Any], key: str) -> Any:
    v = args.get(key)
    if v is None:
        raise ToolError(f"Missing required argument: {key}")
    return v


def _opt_str(args: Dict[str, Any], key: str) -> Optional[str]:
    v = args.get(key)
    return None if v is None else str(v)


def build_tools(app) -> List[Tool]:
    ctx = app.context
    gq = app.graph_query

    def stack_trace(args):
        raw = _require(args, "stackTrace")
        if not isinstance(raw, list):
            raise ToolError("stackTrace must be an array of frames")
        frames = []
        for f in raw:
            if not isinstance(f, dict):
                continue
            ln = f.get("lineNumber")
            frames.append({"className": f.get("className"), "methodName": f.get("methodName"),
                           "lineNumber": int(ln) if isinstance(ln, (int, float)) and not isinstance(ln, bool) else None})
        return ctx.get_stack_trace_context(frames)

    return [
        Tool("list_projects",
             "List all indexed projects. Use this to check which repositories have been analyzed and are "
             "available for Datadog stack trace correlation. Includes project description derived from README.",
             {"type": "object", "properties": {}},
             lambda a: ctx.list_projects()),
        Tool("get_class_context",
             "Get business context for a Java class by its fully qualified name. Returns class type, "
             "description, all methods, and project description from README. Use this when Datadog shows an "
             "error in a specific class to understand its purpose and behavior.",
             {"type": "object", "properties": {"className": _CLASS_NAME,
                                               "projectName": {"type": "string", "description": _PROJECT_SCOPE}},
              "required": ["className"]},
             lambda a: ctx.get_class_context(str(_require(a, "className")), _opt_str(a, "projectName"))),
        Tool("get_method_context",
             "Get detailed context for a specific method, including business logic, dependencies, exceptions, "
             "HTTP endpoint info, and project description from README. Use this when Datadog shows an error in "
             "a specific method to understand what it does and why it might fail.",
             {"type": "object", "properties": {"className": _CLASS_NAME,
                                               "methodName": {"type": "string", "description": "The method name"},
                                               "projectName": {"type": "string", "description": _PROJECT_SCOPE}},
              "required": ["className", "methodName"]},
             lambda a: ctx.get_method_context(str(_require(a, "className")), str(_require(a, "methodName")),
                                              _opt_str(a, "projectName"))),
        Tool("get_stack_trace_context",
             "PRIMARY TOOL for Datadog error correlation. Takes a full stack trace (array of "
             "className/methodName/lineNumber frames) and returns business context for each frame, plus project "
             "description from README. Use this IMMEDIATELY after getting error traces or stack traces from "
             "Datadog to understand the execution path and root cause.",
             {"type": "object", "properties": {"stackTrace": {
                 "type": "array", "description": "The stack trace frames",
                 "items": {"type": "object", "properties": {
                     "className": _CLASS_NAME,
                     "methodName": {"type": "string", "description": "The method name"},
                     "lineNumber": {"type": "integer", "description": "The line number in the source file"}},
                     "required": ["className", "methodName"]}}},
              "required": ["stackTrace"]},
             stack_trace),
        Tool("get_class_dependencies",
             "Get the dependency graph around a class. Returns what this class imports (dependencies), what "
             "imports it (dependents), and method parameter types. Use this to understand how a class connects "
             "to the rest of the system.",
             {"type": "object", "properties": {"className": _CLASS_NAME,
                                               "projectName": {"type": "string", "description": _PROJECT_SCOPE}},
              "required": ["className"]},
             lambda a: ctx.get_class_dependencies(str(_require(a, "className")), _opt_str(a, "projectName"))),
        Tool("get_project_overview",
             "Get a structural overview of an indexed project. Returns entry points (controllers, listeners), "
             "HTTP endpoints, class type breakdown, and project description. Use this to understand the "
             "architecture before drilling into specific classes.",
             {"type": "object", "properties": {"projectName": _PROJECT_NAME}, "required": ["projectName"]},
             lambda a: ctx.get_project_overview(str(_require(a, "projectName")))),
        Tool("get_service_api",
             "Get the public API surface of an indexed microservice. Returns all HTTP endpoints grouped by "
             "controller, with parameter types (DTOs), descriptions, business logic, and exceptions. Use this "
             "when you need to integrate with or call another microservice.",
             {"type": "object", "properties": {"projectName": _PROJECT_NAME}, "required": ["projectName"]},
             lambda a: ctx.get_service_api(str(_require(a, "projectName")))),
        Tool("search_project",
             "Search for classes within a specific project by partial name. Returns matching classes with their "
             "type, description, entry point status, and source file. Use this to discover classes in a project "
             "when you don't know the exact fully qualified name.",
             {"type": "object", "properties": {
                 "projectName": _PROJECT_NAME,
                 "query": {"type": "string",
                           "description": "Partial class name or keyword to search for (case-insensitive)"}},
              "required": ["projectName", "query"]},
             lambda a: ctx.search_project(str(_require(a, "projectName")), str(_require(a, "query")))),
        Tool("graph_query",
             "Query the in-memory project graph using a colon-separated DSL. Supports listing endpoints, "
             "classes, and entry points; navigating to any vertex (class) by name; sub-navigation (methods, "
             "dependencies, dependents); projection modifiers (+logic, +dependencies); and existence checks "
             "(?methodName). All queries resolve from memory, no DB access. Examples: order-service:endpoints, "
             "order-service:endpoints:+logic, order-service:UserService:methods, order-service:UserService:?create",
             {"type": "object", "properties": {"query": {
                 "type": "string",
                 "description": "Colon-separated graph query. Syntax: project:target[:navigation]*[:+include]*"
                                "[:?check]. Keywords: endpoints, classes, entrypoints. Examples: "
                                "order-service:endpoints, order-service:endpoints:+logic, "
                                "order-service:UserService:methods:+logic, order-service:UserService:?createUser"}},
              "required": ["query"]},
             lambda a: gq.query(_require(a, "query")).to_dict()),
    ]


class ToolRegistry:
    def __init__(self, app) -> None:
        self.tools = {t.name: t for t in build_tools(app)}

    def list(self) -> List[dict]:
        return [t.spec() for t in self.tools.values()]

    def call(self, name: str, arguments: Optional[Dict[str, Any]]) -> dict:
        """Returns an MCP CallToolResult dict; exceptions become isError results."""
        tool = self.tools.get(name)
        if tool is None:
            raise KeyError(name)
        args = arguments or {}
        try:
            with span(f"tool.{name}"):
                result = tool.handler(args)
            text = json.dumps(result, ensure_ascii=False, separators=(",", ":"), default=str)
            return {"content": [{"type": "text", "text": text}], "isError": False}
        except Exception as e:
            LOG.error("Tool execution error in %s: %s", name, e, exc_info=not isinstance(e, (ToolError, DomainError)))
            return {"content": [{"type": "text", "text": f"Error: {e}"}], "isError": True}
