"""Context read operations behind the MCP tools and REST endpoints.

Parity: the query half of ``analysis/application/CodeContextService.java`` --
``getClassContext`` (``:901-978``), ``getMethodContext`` (``:1000-1088``),
``getClassDependencies`` (``:1113-1198``), ``getProjectOverview``
(``:1211-1276``), ``getServiceApi`` (``:1288-1380``), ``getStackTraceContext``
(``:1392-1446``) with ``resolveNeighbors`` (``:1550-1613``), ``listProjects``
(``:1453-1478``), ``searchProject`` (``:1492-1530``), ``listKnownProjects``
(``:1793-1806``) and the response records (``:1817-2222``).  Responses are
plain dicts whose keys and key order match the reference's Jackson output.

Differences:

* every per-row lookup is batched (``IN (...)``) -- no N+1 queries;
* class lookups for neighbours / dependencies / search matches are scoped to
  the graph's own project instead of a global FQCN lookup that threw on
  duplicates; a global lookup picks the most recently analyzed project;
* ``list_projects`` reads a stored ``base_package`` (computed at analysis)
  instead of loading every class of every project per call;
* stack frames fall back from ``Outer$Inner`` / ``Outer$$Lambda...`` /
  CGLIB proxy names to the outer class and from ``lambda$m$0`` to ``m`` when
  the exact name is not indexed.
"""
from __future__ import annotations

import re
from typing import Any, Dict, Iterable, List, Optional, Sequence

from ..graph.cache import GraphCache
from ..graph.project_graph import ProjectGraph
from ..models.domain import Project, SourceClass, SourceMethod
from ..store.repositories import Repositories, to_iso

PROJECT_NOT_FOUND_MSG = "Project not found. Use list_projects to see available projects."


def _simple(fqcn: str) -> str:
    i = fqcn.rfind(".")
    return fqcn[i + 1:] if i >= 0 else fqcn


_LAMBDA_RE = re.compile(r"^lambda\$(.+?)\$\d+$")


def candidate_class_names(name: str) -> List[str]:
    out = [name]
    if "$" in name:
        out.append(name.split("$", 1)[0])
    return out


def candidate_method_names(name: Optional[str]) -> List[Optional[str]]:
    if not name:
        return [name]
    out = [name]
    m = _LAMBDA_RE.match(name)
    if m:
        out.append(m.group(1))
    if name in ("<init>", "<clinit>"):
        out.append(None)
    return out


class ContextService:
    def __init__(self, repos: Repositories, cache: GraphCache) -> None:
        self.repos = repos
        self.cache = cache

    # ------------------------------------------------------------ helpers
    def _known_projects(self) -> List[dict]:
        out = []
        for p in self.repos.projects.find_all():
            out.append({"name": p.name, "repositoryUrl": p.repository_url.value,
                        "basePackage": self._base_package(p)})
        return out

    def _base_package(self, p: Project) -> Optional[str]:
        if p.base_package is not None:
            return p.base_package
        from ..index.pipeline import common_package_prefix
        pkgs = self.repos.classes.package_names(p.id)
        if not pkgs:
            return None
        return common_package_prefix(pkgs)

    @staticmethod
    def _project_meta(p: Optional[Project]):
        return (p.repository_url.value if p else None, p.description if p else None)

    @staticmethod
    def _method_summary(m: SourceMethod) -> dict:
        return {"name": m.method_name, "description": m.description, "businessLogic": list(m.business_logic)}

    @staticmethod
    def _entry(order: int, sc: SourceClass, m: SourceMethod) -> dict:
        return {"order": order, "className": sc.full_class_name, "methodName": m.method_name,
                "classType": sc.class_type.value, "description": m.description,
                "businessLogic": list(m.business_logic), "httpEndpoint": m.http_endpoint(), "found": True}

    # ---------------------------------------------------------- list_projects
    def list_projects(self) -> List[dict]:
        counts = self.repos.classes.count_by_project()
        endpoints = self.repos.methods.count_endpoints_by_project()
        out = []
        for p in self.repos.projects.find_all():
            out.append({"id": p.id, "name": p.name, "repositoryUrl": p.repository_url.value,
                        "basePackage": self._base_package(p), "description": p.description,
                        "status": p.status.value, "lastAnalyzedAt": to_iso(p.last_analyzed_at),
                        "classCount": counts.get(p.id, 0), "endpointCount": endpoints.get(p.id, 0)})
        return out

    # --------------------------------------------------------- search_project
    def search_project(self, project_name: str, query: str) -> dict:
        graph = self.cache.get_graph_by_project_name(project_name)
        if graph is None:
            return {"found": False, "projectName": project_name, "query": query, "matches": [],
                    "totalClassesInProject": 0, "message": PROJECT_NOT_FOUND_MSG}
        q = (query or "").lower()
        ids = [i for i in graph.identifiers() if q in i.lower() or q in _simple(i).lower()]
        pid = self.cache.get_project_id_by_name(project_name)
        classes = self.repos.classes.find_by_full_class_names(ids, project_id=pid)
        matches = []
        for ident in ids:
            sc = classes.get(ident)
            matches.append({"className": ident, "classType": sc.class_type.value if sc else None,
                            "description": sc.description if sc else None,
                            "entryPoint": graph.is_entry_point(ident), "sourceFile": graph.source_file(ident)})
        return {"found": True, "projectName": project_name, "query": query, "matches": matches,
                "totalClassesInProject": graph.node_count(), "message": None}

    # ------------------------------------------------------ get_class_context
    @staticmethod
    def _class_not_found(name: str, known: List[dict]) -> dict:
        return {"found": False, "className": name, "classType": None, "description": None,
                "projectDescription": None, "methods": [], "projectUrl": None,
                "message": "No context available for this class", "knownProjects": known, "graphInfo": None}

    def _locate(self, class_name: str, project_name: Optional[str]):
        """Returns (SourceClass | None, graph | None, miss_reason)."""
        if project_name is not None:
            graph = self.cache.get_graph_by_project_name(project_name)
            if graph is None or not graph.contains(class_name):
                return None, graph, "missing"
            pid = self.cache.get_project_id_by_name(project_name)
            sc = self.repos.classes.find_by_project_id_and_full_class_name(pid, class_name)
            return sc, graph, None if sc else "missing"
        sc = self.repos.classes.find_by_full_class_name(class_name)
        if sc is None:
            return None, None, "missing"
        return sc, self.cache.get_graph(sc.project_id), None

    def get_class_context(self, class_name: str, project_name: Optional[str] = None) -> dict:
        sc, graph, miss = self._locate(class_name, project_name)
        if sc is None:
            return self._class_not_found(class_name, self._known_projects())
        methods = self.repos.methods.find_by_class_id(sc.id)
        url, desc = self._project_meta(self.repos.projects.find_by_id(sc.project_id))
        graph_info = None
        if graph is not None and graph.contains(class_name):
            graph_info = {"dependencies": list(graph.dependencies(class_name)),
                          "dependents": list(graph.dependents(class_name)),
                          "entryPoint": graph.is_entry_point(class_name)}
        return {"found": True, "className": sc.full_class_name, "classType": sc.class_type.value,
                "description": sc.description, "projectDescription": desc,
                "methods": [self._method_summary(m) for m in methods], "projectUrl": url, "message": None,
                "knownProjects": [], "graphInfo": graph_info}

    # ----------------------------------------------------- get_method_context
    @staticmethod
    def _method_not_found(cls_name: str, method: str, known: List[dict], message: str) -> dict:
        return {"found": False, "className": cls_name, "methodName": method, "httpEndpoint": None,
                "description": None, "projectDescription": None, "businessLogic": [], "exceptions": [],
                "sourceFile": None, "lineNumber": None, "projectUrl": None, "message": message,
                "knownProjects": known, "parameterTypes": []}

    def get_method_context(self, class_name: str, method_name: str, project_name: Optional[str] = None) -> dict:
        sc, graph, miss = self._locate(class_name, project_name)
        if sc is None:
            return self._method_not_found(class_name, method_name, self._known_projects(),
                                          "No context available for this method")
        m = self.repos.methods.find_by_class_id_and_method_name(sc.id, method_name)
        if m is None:
            return self._method_not_found(class_name, method_name, [], "Class found but method not indexed")
        url, desc = self._project_meta(self.repos.projects.find_by_id(sc.project_id))
        params = []
        if graph is not None:
            links = graph.method_parameters(class_name).get(method_name, ())
            params = [{"position": l.position, "typeName": l.target_identifier} for l in links]
        return {"found": True, "className": sc.full_class_name, "methodName": m.method_name,
                "httpEndpoint": m.http_endpoint(), "description": m.description, "projectDescription": desc,
                "businessLogic": list(m.business_logic), "exceptions": list(m.exceptions),
                "sourceFile": sc.source_file, "lineNumber": m.line_number, "projectUrl": url, "message": None,
                "knownProjects": [], "parameterTypes": params}

    # ------------------------------------------------ get_stack_trace_context
    def get_stack_trace_context(self, frames: Sequence[dict]) -> dict:
        frames = [f for f in frames if isinstance(f, dict)]
        names = []
        for f in frames:
            names.extend(candidate_class_names(str(f.get("className") or "")))
        classes = self.repos.classes.find_by_full_class_names(names)
        entries: List[dict] = []
        missing: List[dict] = []
        project_url = project_desc = project_id = None
        # every frame's class methods in one query (reference: one per frame)
        methods_cache: Dict[str, List[SourceMethod]] = self.repos.methods.find_by_class_ids(
            list({sc.id for sc in classes.values()}))
        order = 1
        for f in frames:
            cname = str(f.get("className") or "")
            mname = f.get("methodName")
            frame = {"className": cname, "methodName": mname, "lineNumber": f.get("lineNumber")}
            sc = next((classes[c] for c in candidate_class_names(cname) if c in classes), None)
            if sc is None:
                missing.append(frame)
                entries.append({"order": order, "className": cname, "methodName": mname, "classType": None,
                                "description": None, "businessLogic": [], "httpEndpoint": None, "found": False})
                order += 1
                continue
            ms = methods_cache.get(sc.id) or []
            method = None
            for cand in candidate_method_names(mname):
                if cand is None:
                    cand = _simple(sc.full_class_name)  # constructor frame
                method = next((m for m in ms if m.method_name == cand), None)
                if method is not None:
                    break
            if method is None:
                missing.append(frame)
                entries.append({"order": order, "className": cname, "methodName": mname,
                                "classType": sc.class_type.value, "description": None, "businessLogic": [],
                                "httpEndpoint": None, "found": False})
                order += 1
                continue
            if project_url is None:
                project_url, project_desc = self._project_meta(self.repos.projects.find_by_id(sc.project_id))
                project_id = sc.project_id
            e = self._entry(order, sc, method)
            e["className"] = cname if cname == sc.full_class_name else sc.full_class_name
            entries.append(e)
            order += 1
        related = self._resolve_neighbors(entries, project_id)
        return {"executionPath": entries, "missingContext": missing, "projectUrl": project_url,
                "projectDescription": project_desc, "relatedDependencies": related}

    def _resolve_neighbors(self, entries: List[dict], project_id: Optional[str]) -> List[dict]:
        if project_id is None:
            return []
        graph = self.cache.get_graph(project_id)
        if graph is None:
            return []
        matched: Dict[str, None] = {}
        for e in entries:
            if e["found"]:
                matched[e["className"]] = None
        neighbors: Dict[str, None] = {}
        for c in matched:
            for n in graph.resolve(c):
                if n not in matched:
                    neighbors[n] = None
        classes = self.repos.classes.find_by_full_class_names(list(neighbors), project_id=project_id)
        methods = self.repos.methods.find_by_class_ids([classes[n].id for n in neighbors if n in classes])
        out: List[dict] = []
        order = 1
        for n in neighbors:
            sc = classes.get(n)
            if sc is None:
                continue
            ms = methods.get(sc.id) or []
            if not ms:
                out.append({"order": order, "className": sc.full_class_name, "methodName": None,
                            "classType": sc.class_type.value, "description": sc.description,
                            "businessLogic": [], "httpEndpoint": None, "found": True})
                order += 1
            else:
                for m in ms:
                    out.append(self._entry(order, sc, m))
                    order += 1
        return out

    # ------------------------------------------------- get_class_dependencies
    @staticmethod
    def _deps_result(found: bool, name: str, entry: bool, deps, dependents, mparams, message) -> dict:
        return {"found": found, "className": name, "entryPoint": entry, "dependencies": deps,
                "dependents": dependents, "methodParameterTypes": mparams, "message": message}

    def get_class_dependencies(self, class_name: str, project_name: Optional[str] = None) -> dict:
        if project_name is not None:
            graph = self.cache.get_graph_by_project_name(project_name)
            if graph is None:
                return self._deps_result(False, class_name, False, [], [], [], PROJECT_NOT_FOUND_MSG)
            if not graph.contains(class_name):
                return self._deps_result(False, class_name, False, [], [], [],
                                         f"Class not found in project {project_name}")
            return self._build_deps(class_name, graph, self.cache.get_project_id_by_name(project_name))
        sc = self.repos.classes.find_by_full_class_name(class_name)
        if sc is None:
            return self._deps_result(False, class_name, False, [], [], [], "Class not found in any indexed project")
        graph = self.cache.get_graph(sc.project_id)
        if graph is None or not graph.contains(class_name):
            return self._deps_result(False, class_name, False, [], [], [],
                                     "No graph data available for this project")
        return self._build_deps(class_name, graph, sc.project_id)

    def _build_deps(self, name: str, graph: ProjectGraph, project_id: Optional[str]) -> dict:
        deps = list(graph.dependencies(name))
        dependents = list(graph.dependents(name))
        params = graph.method_parameters(name)
        wanted = deps + dependents + [l.target_identifier for ls in params.values() for l in ls]
        classes = self.repos.classes.find_by_full_class_names(wanted, project_id=project_id)

        def summary(c: str) -> dict:
            sc = classes.get(c)
            return {"className": c, "classType": sc.class_type.value if sc else None,
                    "description": sc.description if sc else None}

        mp = [{"methodName": m, "parameterTypes": [summary(l.target_identifier) for l in links]}
              for m, links in params.items()]
        return self._deps_result(True, name, graph.is_entry_point(name), [summary(d) for d in deps],
                                 [summary(d) for d in dependents], mp, None)

    # --------------------------------------------------- get_project_overview
    def get_project_overview(self, project_name: str) -> dict:
        p = self.repos.projects.find_by_name(project_name)
        if p is None:
            return {"found": False, "projectName": project_name, "repositoryUrl": None, "description": None,
                    "totalClasses": 0, "totalEntryPoints": 0, "classTypeBreakdown": {}, "entryPoints": [],
                    "message": PROJECT_NOT_FOUND_MSG}
        breakdown = self.repos.classes.class_type_breakdown(p.id)
        total = sum(breakdown.values())
        graph = self.cache.get_graph(p.id)
        if graph is None:
            return {"found": True, "projectName": p.name, "repositoryUrl": p.repository_url.value,
                    "description": p.description, "totalClasses": total, "totalEntryPoints": 0,
                    "classTypeBreakdown": breakdown, "entryPoints": [], "message": "No graph data available"}
        eps = list(graph.entry_points())
        classes = self.repos.classes.find_by_full_class_names(eps, project_id=p.id)
        methods = self.repos.methods.find_by_class_ids([c.id for c in classes.values()])
        summaries = []
        for ep in eps:
            sc = classes.get(ep)
            if sc is None:
                continue
            summaries.append({"className": sc.full_class_name, "classType": sc.class_type.value,
                              "description": sc.description,
                              "httpEndpoints": [m.http_endpoint() for m in methods.get(sc.id, [])
                                                if m.is_http_endpoint()]})
        return {"found": True, "projectName": p.name, "repositoryUrl": p.repository_url.value,
                "description": p.description, "totalClasses": total, "totalEntryPoints": len(eps),
                "classTypeBreakdown": breakdown, "entryPoints": summaries, "message": None}

    # -------------------------------------------------------- get_service_api
    def get_service_api(self, project_name: str) -> dict:
        p = self.repos.projects.find_by_name(project_name)
        if p is None:
            return {"found": False, "projectName": project_name, "repositoryUrl": None, "description": None,
                    "controllers": [], "message": PROJECT_NOT_FOUND_MSG}
        graph = self.cache.get_graph(p.id)
        if graph is None:
            return {"found": False, "projectName": project_name, "repositoryUrl": p.repository_url.value,
                    "description": p.description, "controllers": [],
                    "message": "No graph data available for this project. The project may need to be re-analyzed."}
        eps = list(graph.entry_points())
        param_targets = []
        for ep in eps:
            for links in graph.method_parameters(ep).values():
                param_targets.extend(l.target_identifier for l in links)
        classes = self.repos.classes.find_by_full_class_names(eps + param_targets, project_id=p.id)
        methods = self.repos.methods.find_by_class_ids([classes[e].id for e in eps if e in classes])
        controllers = []
        for ep in eps:
            sc = classes.get(ep)
            if sc is None:
                continue
            cparams = graph.method_parameters(ep)
            endpoints = []
            for m in methods.get(sc.id, []):
                if not m.is_http_endpoint():
                    continue
                plist = []
                for link in cparams.get(m.method_name, ()):
                    pc = classes.get(link.target_identifier)
                    plist.append({"position": link.position, "className": link.target_identifier,
                                  "classType": pc.class_type.value if pc else None,
                                  "description": pc.description if pc else None})
                endpoints.append({"methodName": m.method_name, "httpMethod": m.http_method,
                                  "httpPath": m.http_path, "description": m.description,
                                  "businessLogic": list(m.business_logic), "exceptions": list(m.exceptions),
                                  "parameters": plist})
            if endpoints:
                controllers.append({"className": sc.full_class_name, "description": sc.description,
                                    "endpoints": endpoints})
        return {"found": True, "projectName": p.name, "repositoryUrl": p.repository_url.value,
                "description": p.description, "controllers": controllers, "message": None}
