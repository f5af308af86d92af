"""Graph query DSL: ``project:target[:navigation]*[:+include]*[:?check]``.

Parity: ``analysis/application/GraphQuery.java`` (lexer, ``parse`` ``:95-163``;
helpers ``:185-289``) and ``GraphQueryService.java`` (executor ``:53-475``).
Queries are answered purely from the in-memory graph cache -- no database.

Semantics kept exactly: Java ``String.split(":")`` drops trailing empty
segments; segment prefixes ``+`` (INCLUDE) and ``?`` (CHECK); keywords
``endpoints`` / ``classes`` / ``entrypoints``; vertex resolution exact id ->
case-insensitive simple name -> case-insensitive substring; a CHECK wins over
sub-navigation; sub-navigations ``methods`` / ``dependencies`` / ``dependents``
/ ``method:<name>``; anything else -> overview.  Result
``{resultType, project, count, results[]}``.
"""
from __future__ import annotations

import enum
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Tuple

from ..graph.cache import GraphCache
from ..graph.project_graph import MethodInfo, ProjectGraph
from ..utils.errors import DomainError


class TokenType(enum.Enum):
    NAVIGATE = "NAVIGATE"
    INCLUDE = "INCLUDE"
    CHECK = "CHECK"


@dataclass(frozen=True)
class Token:
    type: TokenType
    value: str

    def __str__(self) -> str:
        if self.type is TokenType.INCLUDE:
            return "+" + self.value
        if self.type is TokenType.CHECK:
            return "?" + self.value
        return self.value


def _java_split_colon(s: str) -> List[str]:
    parts = s.split(":")
    while parts and parts[-1] == "":
        parts.pop()
    return parts


class GraphQuery:
    __slots__ = ("raw", "project", "tokens")

    def __init__(self, raw: str, project: str, tokens: Tuple[Token, ...]) -> None:
        self.raw = raw
        self.project = project
        self.tokens = tokens

    @classmethod
    def parse(cls, query: Optional[str]) -> "GraphQuery":
        if query is None or not str(query).strip():
            raise DomainError("Query is required", "INVALID_QUERY")
        trimmed = str(query).strip()
        parts = _java_split_colon(trimmed)
        if len(parts) < 2:
            raise DomainError(f"Query must have at least project:target. Got: {trimmed}", "INVALID_QUERY")
        project = parts[0].strip()
        if not project:
            raise DomainError("Project name is required", "INVALID_QUERY")
        tokens: List[Token] = []
        for seg in parts[1:]:
            seg = seg.strip()
            if not seg:
                continue
            if seg[0] == "+":
                v = seg[1:].strip()
                if not v:
                    raise DomainError("Include modifier (+) requires a value", "INVALID_QUERY")
                tokens.append(Token(TokenType.INCLUDE, v))
            elif seg[0] == "?":
                v = seg[1:].strip()
                if not v:
                    raise DomainError("Check (?) requires a value", "INVALID_QUERY")
                tokens.append(Token(TokenType.CHECK, v))
            else:
                tokens.append(Token(TokenType.NAVIGATE, seg))
        if not tokens:
            raise DomainError("Query must have at least one target after project", "INVALID_QUERY")
        if tokens[0].type is not TokenType.NAVIGATE:
            raise DomainError("First segment after project must be a navigation target, not a modifier. "
                              f"Got: {tokens[0]}", "INVALID_QUERY")
        return cls(trimmed, project, tuple(tokens))

    def navigations(self) -> List[Token]:
        return [t for t in self.tokens if t.type is TokenType.NAVIGATE]

    def first_navigation(self) -> Optional[str]:
        for t in self.tokens:
            if t.type is TokenType.NAVIGATE:
                return t.value
        return None

    def navigations_from(self, index: int) -> List[str]:
        navs = self.navigations()
        return [t.value for t in navs[index:]] if index < len(navs) else []

    def includes(self) -> List[Token]:
        return [t for t in self.tokens if t.type is TokenType.INCLUDE]

    def has_include(self, value: str) -> bool:
        v = value.lower()
        return any(t.type is TokenType.INCLUDE and t.value.lower() == v for t in self.tokens)

    def checks(self) -> List[Token]:
        return [t for t in self.tokens if t.type is TokenType.CHECK]

    def has_check(self) -> bool:
        return any(t.type is TokenType.CHECK for t in self.tokens)

    def check_value(self) -> Optional[str]:
        for t in self.tokens:
            if t.type is TokenType.CHECK:
                return t.value
        return None


@dataclass
class GraphQueryResult:
    result_type: str
    project: str
    count: int
    results: List[Dict[str, Any]]

    def to_dict(self) -> dict:
        return {"resultType": self.result_type, "project": self.project, "count": self.count,
                "results": self.results}


def _simple(fqcn: str) -> str:
    i = fqcn.rfind(".")
    return fqcn[i + 1:] if i >= 0 else fqcn


class GraphQueryService:
    def __init__(self, cache: GraphCache) -> None:
        self.cache = cache

    def query(self, text: str) -> GraphQueryResult:
        return self.execute(GraphQuery.parse(text))

    def execute(self, q: GraphQuery) -> GraphQueryResult:
        graph = self.cache.get_graph_by_project_name(q.project)
        if graph is None:
            raise DomainError(f"Project not found: {q.project}. Use list_projects to see available projects.",
                              "PROJECT_NOT_FOUND")
        target = q.first_navigation() or ""
        t = target.lower()
        if t == "endpoints":
            return self._endpoints(q, graph)
        if t == "classes":
            return self._classes(q, graph)
        if t == "entrypoints":
            return self._entrypoints(q, graph)
        return self._vertex(q, graph, target)

    # ----------------------------------------------------------- keywords
    def _endpoints(self, q: GraphQuery, g: ProjectGraph) -> GraphQueryResult:
        logic = q.has_include("logic")
        out = []
        for ident, mi in g.all_endpoints():
            ni = g.node_info(ident)
            item = {"className": ident, "classType": ni.class_type if ni else None,
                    "methodName": mi.method_name, "httpMethod": mi.http_method,
                    "httpPath": mi.http_path, "description": mi.description}
            if logic:
                item["businessLogic"] = list(mi.business_logic)
            out.append(item)
        return GraphQueryResult("endpoints", q.project, len(out), out)

    def _classes(self, q: GraphQuery, g: ProjectGraph) -> GraphQueryResult:
        deps, dependents, methods = q.has_include("dependencies"), q.has_include("dependents"), q.has_include("methods")
        out = []
        for ident in g.identifiers():
            ni = g.node_info(ident)
            item = {"className": ident, "classType": ni.class_type if ni else None,
                    "description": ni.description if ni else None, "sourceFile": g.source_file(ident),
                    "entryPoint": g.is_entry_point(ident)}
            if deps:
                item["dependencies"] = list(g.dependencies(ident))
            if dependents:
                item["dependents"] = list(g.dependents(ident))
            if methods:
                item["methods"] = self._summaries(ident, g, False)
            out.append(item)
        return GraphQueryResult("classes", q.project, len(out), out)

    def _entrypoints(self, q: GraphQuery, g: ProjectGraph) -> GraphQueryResult:
        logic = q.has_include("logic")
        out = []
        for ep in g.entry_points():
            ni = g.node_info(ep)
            eps = []
            for mi in g.methods(ep):
                if mi.is_http_endpoint():
                    m = {"methodName": mi.method_name, "httpEndpoint": mi.http_endpoint(),
                         "description": mi.description}
                    if logic:
                        m["businessLogic"] = list(mi.business_logic)
                    eps.append(m)
            out.append({"className": ep, "classType": ni.class_type if ni else None,
                        "description": ni.description if ni else None, "endpoints": eps})
        return GraphQueryResult("entrypoints", q.project, len(out), out)

    # ------------------------------------------------------------- vertex
    def _vertex(self, q: GraphQuery, g: ProjectGraph, target: str) -> GraphQueryResult:
        ident = self.resolve_class_name(target, g)
        if ident is None:
            raise DomainError(f"Class not found: {target} in project {q.project}", "CLASS_NOT_FOUND")
        if q.has_check():
            return self._check(ident, q, g)
        subs = q.navigations_from(1)
        if not subs:
            return self._overview(ident, g, q)
        nav = subs[0].lower()
        if nav == "methods":
            return self._methods(ident, g, q)
        if nav == "dependencies":
            return self._deps(ident, g, q, True)
        if nav == "dependents":
            return self._deps(ident, g, q, False)
        if nav == "method":
            if len(subs) < 2:
                raise DomainError("Method name required. Example: project:Foo:method:bar", "INVALID_QUERY")
            return self._single_method(ident, g, q, subs[1])
        return self._overview(ident, g, q)

    def _overview(self, ident: str, g: ProjectGraph, q: GraphQuery) -> GraphQueryResult:
        ni = g.node_info(ident)
        item = {"className": ident, "classType": ni.class_type if ni else None,
                "description": ni.description if ni else None, "sourceFile": g.source_file(ident),
                "entryPoint": g.is_entry_point(ident), "dependencies": list(g.dependencies(ident)),
                "dependents": list(g.dependents(ident)),
                "methods": self._summaries(ident, g, q.has_include("logic"))}
        return GraphQueryResult("class", q.project, 1, [item])

    def _methods(self, ident: str, g: ProjectGraph, q: GraphQuery) -> GraphQueryResult:
        logic = q.has_include("logic")
        out = []
        for mi in g.methods(ident):
            item: Dict[str, Any] = {"methodName": mi.method_name, "description": mi.description}
            if logic:
                item["businessLogic"] = list(mi.business_logic)
            item["exceptions"] = list(mi.exceptions)
            if mi.is_http_endpoint():
                item["httpMethod"] = mi.http_method
                item["httpPath"] = mi.http_path
            if mi.line_number is not None:
                item["lineNumber"] = mi.line_number
            out.append(item)
        return GraphQueryResult("methods", q.project, len(out), out)

    def _deps(self, ident: str, g: ProjectGraph, q: GraphQuery, outgoing: bool) -> GraphQueryResult:
        related = g.dependencies(ident) if outgoing else g.dependents(ident)
        out = []
        for d in related:
            ni = g.node_info(d)
            out.append({"className": d, "classType": ni.class_type if ni else None,
                        "description": ni.description if ni else None, "sourceFile": g.source_file(d)})
        return GraphQueryResult("dependencies" if outgoing else "dependents", q.project, len(out), out)

    def _single_method(self, ident: str, g: ProjectGraph, q: GraphQuery, name: str) -> GraphQueryResult:
        want = name.lower()
        for mi in g.methods(ident):
            if mi.method_name.lower() == want:
                item: Dict[str, Any] = {"className": ident, "methodName": mi.method_name,
                                        "description": mi.description,
                                        "businessLogic": list(mi.business_logic),
                                        "exceptions": list(mi.exceptions)}
                if mi.is_http_endpoint():
                    item["httpMethod"] = mi.http_method
                    item["httpPath"] = mi.http_path
                if mi.line_number is not None:
                    item["lineNumber"] = mi.line_number
                return GraphQueryResult("method", q.project, 1, [item])
        raise DomainError(f"Method not found: {name} in class {ident}", "METHOD_NOT_FOUND")

    def _check(self, ident: str, q: GraphQuery, g: ProjectGraph) -> GraphQueryResult:
        value = q.check_value() or ""
        want = value.lower()
        match: Optional[MethodInfo] = next((m for m in g.methods(ident) if m.method_name.lower() == want), None)
        item: Dict[str, Any] = {"className": ident, "check": value, "exists": match is not None}
        if match is not None:
            item["methodName"] = match.method_name
            item["description"] = match.description
            if match.is_http_endpoint():
                item["httpEndpoint"] = match.http_endpoint()
        return GraphQueryResult("check", q.project, 1, [item])

    # ------------------------------------------------------------ helpers
    @staticmethod
    def _summaries(ident: str, g: ProjectGraph, logic: bool) -> List[dict]:
        out = []
        for mi in g.methods(ident):
            m: Dict[str, Any] = {"methodName": mi.method_name, "description": mi.description}
            if mi.is_http_endpoint():
                m["httpEndpoint"] = mi.http_endpoint()
            if logic:
                m["businessLogic"] = list(mi.business_logic)
            out.append(m)
        return out

    @staticmethod
    def resolve_class_name(name: str, g: ProjectGraph) -> Optional[str]:
        """Exact id -> case-insensitive simple name -> case-insensitive substring."""
        if g.contains(name):
            return name
        low = name.lower()
        for ident in g.identifiers():
            if _simple(ident).lower() == low:
                return ident
        for ident in g.identifiers():
            if low in ident.lower():
                return ident
        return None
