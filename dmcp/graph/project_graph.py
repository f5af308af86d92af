"""Language-agnostic in-memory dependency graph of one project.

Behavioural parity with ``analysis/domain/ProjectGraph.java`` (records
``:44-86``, ``addNode`` ``:160``, ``addDependency`` ``:175-183``,
``markAsEntryPoint`` ``:190-197``, ``addMethodParameter`` ``:212-235``,
``resolve`` ``:359-378``, ``analysisOrder`` ``:390-421``, ``applyEnrichment``
``:558-588``, ``allEndpoints`` ``:606-618``, ``toJson``/``fromJson``
``:634-905``).  Design differences:

* a **reverse adjacency index** makes ``dependents`` O(deg) instead of the
  reference's O(E) scan of every edge set (``:316-328``), so
  ``classes:+dependents`` is O(N+E) rather than O(N*E);
* an endpoint index keeps ``all_endpoints`` proportional to endpoints;
* graphs are **frozen on publish** (:meth:`freeze`): the cache only ever holds
  immutable graphs, which makes concurrent readers safe by construction;
* every ordered collection is insertion-ordered (the reference leaks Java
  ``HashMap`` iteration order into its JSON and query results).

The JSON wire format is the reference's (``nodes``/``edges``/``entryPoints``/
``methodParameters``/``nodeInfo``/``methodInfo``) plus a ``version`` key, and
``from_json`` accepts the old format without the metadata sections.
"""
from __future__ import annotations

import json
from collections import deque
from typing import Dict, Iterable, List, Mapping, NamedTuple, Optional, Tuple

from ..utils.errors import require_non_blank, require_non_negative

GRAPH_JSON_VERSION = 2

_ENCODER: list = []


def _native_encoder():
    if not _ENCODER:
        try:
            from .. import _srcscan  # type: ignore
            _ENCODER.append(getattr(_srcscan, "graph_json", None))
        except ImportError:
            _ENCODER.append(None)
    return _ENCODER[0]


# Value records are NamedTuples: immutable, hashable and ~5x cheaper to build
# than frozen dataclasses on the indexing hot path (10^4-10^5 per project).
class MethodParameterLink(NamedTuple):
    position: int
    target_identifier: str


class NodeInfo(NamedTuple):
    class_type: Optional[str]
    description: Optional[str]


class MethodInfo(NamedTuple):
    method_name: str
    description: Optional[str] = None
    business_logic: Tuple[str, ...] = ()
    exceptions: Tuple[str, ...] = ()
    http_method: Optional[str] = None
    http_path: Optional[str] = None
    line_number: Optional[int] = None

    def is_http_endpoint(self) -> bool:
        return self.http_method is not None and self.http_path is not None

    def http_endpoint(self) -> Optional[str]:
        if not self.is_http_endpoint():
            return None
        return f"{self.http_method} {self.http_path}"


class MethodEnrichmentData(NamedTuple):
    description: Optional[str]
    business_logic: Tuple[str, ...] = ()


class FrozenGraphError(RuntimeError):
    """Raised when a published (frozen) graph is mutated."""


class ProjectGraph:
    __slots__ = ("_nodes", "_out", "_in", "_entry", "_class_ids", "_mparams",
                 "_node_info", "_method_info", "_frozen")

    def __init__(self) -> None:
        self._nodes: Dict[str, str] = {}
        self._out: Dict[str, Dict[str, None]] = {}
        self._in: Dict[str, Dict[str, None]] = {}
        self._entry: Dict[str, None] = {}
        self._class_ids: Dict[str, str] = {}
        self._mparams: Dict[str, Dict[str, List[MethodParameterLink]]] = {}
        self._node_info: Dict[str, NodeInfo] = {}
        self._method_info: Dict[str, List[MethodInfo]] = {}
        self._frozen = False

    # ------------------------------------------------------------------ life
    def freeze(self) -> "ProjectGraph":
        self._frozen = True
        return self

    @property
    def frozen(self) -> bool:
        return self._frozen

    def _check_mutable(self) -> None:
        if self._frozen:
            raise FrozenGraphError("ProjectGraph is frozen (published); copy() it to modify")

    def copy(self) -> "ProjectGraph":
        g = ProjectGraph()
        g._nodes = dict(self._nodes)
        g._out = {k: dict(v) for k, v in self._out.items()}
        g._in = {k: dict(v) for k, v in self._in.items()}
        g._entry = dict(self._entry)
        g._class_ids = dict(self._class_ids)
        g._mparams = {c: {m: list(ls) for m, ls in per.items()} for c, per in self._mparams.items()}
        g._node_info = dict(self._node_info)
        g._method_info = {k: list(v) for k, v in self._method_info.items()}
        return g

    # ------------------------------------------------------------- structure
    def add_node(self, identifier: str, source_file: str) -> None:
        require_non_blank(identifier, "Identifier is required")
        require_non_blank(source_file, "Source file is required")
        self._check_mutable()
        self._nodes[identifier] = source_file

    def add_dependency(self, from_id: str, to_id: str) -> None:
        require_non_blank(from_id, "From identifier is required")
        require_non_blank(to_id, "To identifier is required")
        self._check_mutable()
        nodes = self._nodes
        if from_id not in nodes or to_id not in nodes:
            return
        out = self._out.get(from_id)
        if out is None:
            out = self._out[from_id] = {}
        if to_id in out:
            return
        out[to_id] = None
        rev = self._in.get(to_id)
        if rev is None:
            rev = self._in[to_id] = {}
        rev[from_id] = None

    def mark_as_entry_point(self, identifier: str) -> None:
        require_non_blank(identifier, "Entry point identifier is required")
        self._check_mutable()
        if identifier in self._nodes:
            self._entry[identifier] = None

    def add_method_parameter(self, class_identifier: str, method_name: str,
                             position: int, parameter_type_identifier: str) -> None:
        require_non_blank(class_identifier, "Class identifier is required")
        require_non_blank(method_name, "Method name is required")
        require_non_negative(position, "Position must be non-negative")
        require_non_blank(parameter_type_identifier, "Parameter type identifier is required")
        self._check_mutable()
        if class_identifier not in self._nodes or parameter_type_identifier not in self._nodes:
            return
        per = self._mparams.setdefault(class_identifier, {})
        per.setdefault(method_name, []).append(
            MethodParameterLink(position, parameter_type_identifier))

    def clear_method_parameters(self, class_identifier: str) -> None:
        self._check_mutable()
        self._mparams.pop(class_identifier, None)

    def method_parameters(self, class_identifier: str) -> Mapping[str, Tuple[MethodParameterLink, ...]]:
        per = self._mparams.get(class_identifier)
        if not per:
            return {}
        return {m: tuple(ls) for m, ls in per.items()}

    def method_parameter_targets(self, class_identifier: str) -> Tuple[str, ...]:
        per = self._mparams.get(class_identifier)
        if not per:
            return ()
        seen: Dict[str, None] = {}
        for links in per.values():
            for link in links:
                seen[link.target_identifier] = None
        return tuple(seen)

    def dependencies(self, identifier: Optional[str]) -> Tuple[str, ...]:
        if identifier is None or identifier not in self._nodes:
            return ()
        return tuple(self._out.get(identifier, ()))

    def dependents(self, identifier: Optional[str]) -> Tuple[str, ...]:
        if identifier is None or identifier not in self._nodes:
            return ()
        return tuple(self._in.get(identifier, ()))

    def is_entry_point(self, identifier: Optional[str]) -> bool:
        return identifier is not None and identifier in self._entry

    def entry_points(self) -> Tuple[str, ...]:
        return tuple(self._entry)

    def resolve(self, identifier: Optional[str]) -> Tuple[str, ...]:
        """Direct neighbourhood: outgoing dependencies, then incoming dependents."""
        if identifier is None or identifier not in self._nodes:
            return ()
        seen: Dict[str, None] = dict.fromkeys(self._out.get(identifier, ()))
        for d in self._in.get(identifier, ()):
            seen[d] = None
        return tuple(seen)

    def analysis_order(self) -> List[str]:
        """BFS from entry points over outgoing edges, then unreachable nodes."""
        if not self._nodes:
            return []
        visited: Dict[str, None] = {}
        queue: deque = deque()
        for ep in self._entry:
            if ep not in visited:
                visited[ep] = None
                queue.append(ep)
        out = self._out
        while queue:
            cur = queue.popleft()
            for dep in out.get(cur, ()):
                if dep not in visited:
                    visited[dep] = None
                    queue.append(dep)
        for ident in self._nodes:
            if ident not in visited:
                visited[ident] = None
        return list(visited)

    def bind_class_id(self, identifier: str, class_id: str) -> None:
        require_non_blank(identifier, "Identifier is required")
        require_non_blank(class_id, "Class ID is required")
        self._check_mutable()
        self._class_ids[identifier] = class_id

    def class_id(self, identifier: Optional[str]) -> Optional[str]:
        return self._class_ids.get(identifier) if identifier is not None else None

    def source_file(self, identifier: Optional[str]) -> Optional[str]:
        return self._nodes.get(identifier) if identifier is not None else None

    def contains(self, identifier: Optional[str]) -> bool:
        return identifier is not None and identifier in self._nodes

    __contains__ = contains

    def node_count(self) -> int:
        return len(self._nodes)

    def edge_count(self) -> int:
        return sum(len(v) for v in self._out.values())

    def entry_point_count(self) -> int:
        return len(self._entry)

    def identifiers(self) -> Tuple[str, ...]:
        return tuple(self._nodes)

    def identifier_set(self):
        """Live read-only membership view (a dict keys view, O(1) ``in``)."""
        return self._nodes.keys()

    # -------------------------------------------------------------- metadata
    def set_node_info(self, identifier: str, class_type: Optional[str],
                      description: Optional[str]) -> None:
        require_non_blank(identifier, "Identifier is required")
        self._check_mutable()
        self._node_info[identifier] = NodeInfo(class_type, description)

    def load_static_metadata(self, class_ids: Mapping[str, str], class_types: Mapping[str, Optional[str]],
                             method_infos: Mapping[str, List[MethodInfo]],
                             method_params: Mapping[str, Mapping[str, Sequence[str]]]) -> None:
        """Phase 1 in one call: class ids, node infos (type, no description),
        method infos and parameter links of every parsed unit.  Equivalent to
        ``bind_class_id`` / ``set_node_info`` / ``set_method_infos`` /
        ``add_method_parameter`` per element (same skipping of links whose
        class or target is not a node), validated once per argument instead
        of per element -- the per-call checks were ~25 % of Phase 1."""
        self._check_mutable()
        nodes = self._nodes
        for ident, cid in class_ids.items():
            if not ident or not cid:
                raise ValueError("Identifier and class ID are required")
            self._class_ids[ident] = cid
        tnew = tuple.__new__  # NamedTuples without the generated __new__ wrapper
        for ident, ct in class_types.items():
            self._node_info[ident] = tnew(NodeInfo, (ct, None))
        for ident, infos in method_infos.items():
            self._method_info[ident] = list(infos)
        for ident, per_method in method_params.items():
            if ident not in nodes:
                continue
            per = None
            for mname, targets in per_method.items():
                links = [tnew(MethodParameterLink, (pos, t)) for pos, t in enumerate(targets) if t in nodes]
                if links:
                    if per is None:
                        per = self._mparams.setdefault(ident, {})
                    per.setdefault(mname, []).extend(links)

    def static_metadata_targets(self) -> tuple:
        """The containers :meth:`load_static_metadata` fills, for a native
        Phase 1 that fills them in place with the same values:
        (class_ids, node_info, method_info, method_params, nodes, NodeInfo,
        MethodParameterLink) -- ``native/srcscan/pymodule.cpp::phase1_rows``."""
        self._check_mutable()
        return (self._class_ids, self._node_info, self._method_info, self._mparams, self._nodes, NodeInfo,
                MethodParameterLink)

    def node_info(self, identifier: Optional[str]) -> Optional[NodeInfo]:
        return self._node_info.get(identifier) if identifier is not None else None

    def add_method_info(self, identifier: str, method_info: MethodInfo) -> None:
        require_non_blank(identifier, "Identifier is required")
        self._check_mutable()
        self._method_info.setdefault(identifier, []).append(method_info)

    def set_method_infos(self, identifier: str, infos: Iterable[MethodInfo]) -> None:
        require_non_blank(identifier, "Identifier is required")
        self._check_mutable()
        self._method_info[identifier] = list(infos)

    def methods(self, identifier: Optional[str]) -> Tuple[MethodInfo, ...]:
        ls = self._method_info.get(identifier) if identifier is not None else None
        return tuple(ls) if ls else ()

    def apply_enrichment(self, identifier: str, class_type: Optional[str],
                         class_description: Optional[str],
                         method_enrichments: Optional[Mapping[str, MethodEnrichmentData]]) -> None:
        self._check_mutable()
        self._node_info[identifier] = NodeInfo(class_type, class_description)
        existing = self._method_info.get(identifier)
        if existing is None or method_enrichments is None:
            return
        updated = []
        for mi in existing:
            e = method_enrichments.get(mi.method_name)
            if e is not None:
                updated.append(MethodInfo(mi.method_name, e.description,
                                          tuple(e.business_logic or ()), mi.exceptions,
                                          mi.http_method, mi.http_path, mi.line_number))
            else:
                updated.append(mi)
        self._method_info[identifier] = updated

    def all_endpoints(self) -> List[Tuple[str, MethodInfo]]:
        return [(ident, mi) for ident, ms in self._method_info.items()
                for mi in ms if mi.is_http_endpoint()]

    def has_metadata(self) -> bool:
        return bool(self._node_info)

    # ---------------------------------------------------------- serialization
    def to_dict(self) -> dict:
        class_ids = self._class_ids
        nodes = {}
        for ident, sf in self._nodes.items():
            n = {"sourceFile": sf}
            cid = class_ids.get(ident)
            if cid is not None:
                n["classId"] = cid
            nodes[ident] = n
        mp = {c: {m: [{"position": l.position, "target": l.target_identifier} for l in ls]
                  for m, ls in per.items()} for c, per in self._mparams.items()}
        ni = {}
        for ident, info in self._node_info.items():
            o = {}
            if info.class_type is not None:
                o["classType"] = info.class_type
            if info.description is not None:
                o["description"] = info.description
            ni[ident] = o
        mi_out = {}
        for ident, ms in self._method_info.items():
            arr = []
            for m in ms:
                o = {"methodName": m.method_name}
                if m.description is not None:
                    o["description"] = m.description
                if m.business_logic:
                    o["businessLogic"] = list(m.business_logic)
                if m.exceptions:
                    o["exceptions"] = list(m.exceptions)
                if m.http_method is not None:
                    o["httpMethod"] = m.http_method
                if m.http_path is not None:
                    o["httpPath"] = m.http_path
                if m.line_number is not None:
                    o["lineNumber"] = m.line_number
                arr.append(o)
            mi_out[ident] = arr
        return {
            "version": GRAPH_JSON_VERSION,
            "nodes": nodes,
            "edges": {k: list(v) for k, v in self._out.items()},
            "entryPoints": list(self._entry),
            "methodParameters": mp,
            "nodeInfo": ni,
            "methodInfo": mi_out,
        }

    def to_json(self) -> str:
        """Compact JSON; written natively straight from the graph's containers
        (``_srcscan.graph_json``, byte-identical) when the extension is built,
        else through :meth:`to_dict` + ``json.dumps``."""
        enc = _native_encoder()
        if enc is not None:
            try:
                return enc(GRAPH_JSON_VERSION, self._nodes, self._class_ids, self._out, self._entry,
                           self._mparams, self._node_info, self._method_info)
            except TypeError:
                pass  # an unexpected value type: the generic encoder handles (or rejects) it
        return json.dumps(self.to_dict(), separators=(",", ":"), ensure_ascii=False)

    @classmethod
    def from_json(cls, text: Optional[str]) -> "ProjectGraph":
        require_non_blank(text, "JSON is required")
        try:
            root = json.loads(text)
        except (ValueError, TypeError) as e:
            raise ValueError(f"Failed to deserialize ProjectGraph: {e}") from e
        if not isinstance(root, dict):
            raise ValueError("Failed to deserialize ProjectGraph: root is not an object")
        return cls.from_dict(root)

    @classmethod
    def from_dict(cls, root: dict) -> "ProjectGraph":
        g = cls()
        nodes = root.get("nodes")
        if isinstance(nodes, dict):
            for ident, val in nodes.items():
                sf = val.get("sourceFile") if isinstance(val, dict) else None
                if sf is None:
                    raise ValueError(f"Failed to deserialize ProjectGraph: node {ident} has no sourceFile")
                g._nodes[ident] = str(sf)
                cid = val.get("classId")
                if cid is not None:
                    g._class_ids[ident] = str(cid)
        edges = root.get("edges")
        if isinstance(edges, dict):
            # Edges are restored verbatim (the reference does not re-filter them).
            for frm, deps in edges.items():
                out = g._out.setdefault(frm, {})
                for d in deps or ():
                    d = str(d)
                    out[d] = None
                    g._in.setdefault(d, {})[frm] = None
        eps = root.get("entryPoints")
        if isinstance(eps, list):
            for ep in eps:
                g._entry[str(ep)] = None
        mp = root.get("methodParameters")
        if isinstance(mp, dict):
            for c, per in mp.items():
                dst = g._mparams.setdefault(c, {})
                for m, links in (per or {}).items():
                    dst[m] = [MethodParameterLink(int(p["position"]), str(p["target"]))
                              for p in (links or ())]
        ni = root.get("nodeInfo")
        if isinstance(ni, dict):
            for ident, val in ni.items():
                val = val or {}
                g._node_info[ident] = NodeInfo(val.get("classType"), val.get("description"))
        mi = root.get("methodInfo")
        if isinstance(mi, dict):
            for ident, arr in mi.items():
                ms = []
                for o in arr or ():
                    ln = o.get("lineNumber")
                    ms.append(MethodInfo(str(o["methodName"]), o.get("description"),
                                         tuple(str(x) for x in o.get("businessLogic") or ()),
                                         tuple(str(x) for x in o.get("exceptions") or ()),
                                         o.get("httpMethod"), o.get("httpPath"),
                                         int(ln) if ln is not None else None))
                g._method_info[ident] = ms
        return g

    def __repr__(self) -> str:
        return (f"ProjectGraph(nodes={len(self._nodes)}, edges={self.edge_count()}, "
                f"entryPoints={len(self._entry)}, frozen={self._frozen})")
