"""Source parsers: the language strategy layer over the native front-ends.

Parity: ``analysis/domain/SourceParser.java`` (template method ``parse`` with
three passes -- nodes, import edges filtered by known identifiers, entry points
-- ``:146-194``; per-file hooks ``inferClassType`` / ``extractMethods`` /
``extractMethodParameters``, ``language()``, ``sourceRoot()``) and the three
concrete strategies ``JavaSourceParser`` / ``NodeJsGraalParser`` /
``GoSourceParser``.

MI355X-host design: the whole project is scanned by the native C++ library
(``native/srcscan``, loaded as :mod:`dmcp._srcscan`) in one parallel call that
reads and analyses every file exactly once and resolves dependencies and
parameter types natively.  The per-file hooks answer from that cached scan, so
the indexing pipeline never re-parses (the reference parses each Java file ~7
times across ``parse`` + phase 1 + phase 2).

If the native module cannot be imported, :func:`native_scan` raises -- there is
deliberately no silent pure-Python fallback for the hot path.
"""
from __future__ import annotations

import json
import logging
import os
import time
from dataclasses import dataclass, field
from typing import Any, Dict, List, Mapping, Optional, Sequence, Set

from ..graph.project_graph import ProjectGraph
from ..models.domain import ClassType, StaticMethodInfo
from ..utils.errors import require_non_null

LOG = logging.getLogger(__name__)

_native = None


def native():
    """Imports (building on first use if needed) the native scanner module."""
    global _native
    if _native is not None:
        return _native
    try:
        from .. import _srcscan  # type: ignore
    except ImportError:
        if os.environ.get("DMCP_NO_AUTOBUILD"):
            raise
        from .. import buildtools
        LOG.warning("native srcscan module missing; building it in-tree")
        buildtools.build_srcscan()
        import importlib
        _srcscan = importlib.import_module("dmcp._srcscan")
    _native = _srcscan
    return _native


def native_scan(root: str, language: str = "auto", threads: int = 0, framework: str = "") -> dict:
    raw = native().scan_project(os.path.abspath(root), language, int(threads), framework)
    return json.loads(raw)


def detect_language(root: str) -> str:
    """``CodeContextService.detectParser`` (:1628-1642): go.mod -> Go; package.json
    without pom.xml/build.gradle(.kts) -> TypeScript; else Java."""
    j = os.path.join
    if os.path.isfile(j(root, "go.mod")):
        return "go"
    if (os.path.isfile(j(root, "package.json")) and not os.path.isfile(j(root, "pom.xml"))
            and not os.path.isfile(j(root, "build.gradle"))
            and not os.path.isfile(j(root, "build.gradle.kts"))):
        return "typescript"
    return "java"


@dataclass
class ParsedUnit:
    """One graph node: a Java class, a TS/JS module or a Go package."""

    identifier: str
    source_file: str
    class_type: ClassType
    entry_point: bool
    methods: List[StaticMethodInfo] = field(default_factory=list)
    deps: List[str] = field(default_factory=list)
    params: Dict[str, List[str]] = field(default_factory=dict)
    files: List[str] = field(default_factory=list)


@dataclass
class ParsedProject:
    language: str
    source_root: str
    framework: Optional[dict]
    module: Optional[str]
    units: Dict[str, ParsedUnit]
    file_to_identifier: Dict[str, str]
    stats: dict
    go_analysis: Optional[Any] = None  # dict, or its JSON text until GoSourceParser.go_analysis() parses it
    # ident -> (class id, [method ids]) of class / method rows the scan already
    # handed to the row writer (scan_tree(rows=...)); Phase 1 binds these ids
    static_row_ids: Optional[dict] = None
    # ms of the scan's parts (isolated: child round trip, decode; objects)
    scan_timing: Optional[dict] = None

    def build_graph(self) -> ProjectGraph:
        """The three-pass build (SourceParser.java:163-188) from the scan."""
        g = ProjectGraph()
        for ident, unit in self.units.items():
            g.add_node(ident, unit.source_file)
        for ident, unit in self.units.items():
            for d in unit.deps:
                g.add_dependency(ident, d)
        for ident, unit in self.units.items():
            if unit.entry_point:
                g.mark_as_entry_point(ident)
        return g

    def identifiers(self) -> List[str]:
        return list(self.units)


def _methods_from(raw: Sequence[dict]) -> List[StaticMethodInfo]:
    out = []
    for m in raw:
        out.append(StaticMethodInfo(m["name"], m.get("line"), m.get("httpMethod"), m.get("httpPath"),
                                    tuple(m.get("exceptions") or ())))
    return out


_CLASS_TYPES: Dict[Optional[str], ClassType] = {}


def _class_type(name: Optional[str]) -> ClassType:
    ct = _CLASS_TYPES.get(name)
    if ct is None:
        ct = _CLASS_TYPES[name] = ClassType.from_string(name)
    return ct


def _add_unit(units: Dict[str, ParsedUnit], lang: str, path: str, ident: str, ct: ClassType, entry: bool,
              methods: List[StaticMethodInfo], deps: List[str], params: Dict[str, List[str]]) -> None:
    u = units.get(ident)
    if u is None or lang != "go":
        # Java / TS: a later file with the same identifier replaces the node
        # (ProjectGraph.addNode overwrite semantics).
        if u is not None:
            del units[ident]
        units[ident] = ParsedUnit(ident, path, ct, entry, methods, deps, params, [path])
    else:
        # Go: every file of a package is the same node; the reference keeps
        # only the last file's methods (GoSourceParser + phase 1), here all
        # files contribute (documented divergence).
        u.source_file = path
        u.methods.extend(methods)
        u.params.update(params)
        u.files.append(path)
        for d in deps:
            if d not in u.deps:
                u.deps.append(d)


def to_parsed_project(doc: dict) -> ParsedProject:
    """From the native scan document: the JSON form (``files`` as objects) or
    the direct-object form of ``scan_sources_objects`` (``files`` as tuples
    ``(path, identifier, classType, entryPoint, package, deps, params,
    methods)`` with ``methods`` already :class:`StaticMethodInfo`)."""
    lang = doc["language"]
    units: Dict[str, ParsedUnit] = {}
    file_to_id: Dict[str, str] = {}
    for f in doc.get("files", []):
        if isinstance(f, tuple):
            path, ident, ct, entry, _pkg, deps, params, methods = f
            file_to_id[path] = ident
            _add_unit(units, lang, path, ident, _class_type(ct), entry, methods, deps, dict(params))
            continue
        ident = f["identifier"]
        path = f["path"]
        file_to_id[path] = ident
        _add_unit(units, lang, path, ident, _class_type(f.get("classType")), bool(f.get("entryPoint")),
                  _methods_from(f.get("methods") or ()), list(f.get("deps") or ()),
                  {k: list(v) for k, v in (f.get("params") or {}).items()})
    # the Go analyzer's package document stays JSON text until someone asks
    # for it (GoSourceParser.go_analysis): the indexing pipeline never does,
    # and parsing it cost a 1,000-file repository ~10 ms per analysis
    go = doc.get("go")
    return ParsedProject(lang, doc.get("sourceRoot", "."), doc.get("framework"), doc.get("module"),
                         units, file_to_id, doc.get("stats") or {}, go)


class SourceParser:
    """Strategy per language; ``parse`` scans natively and caches the result."""

    language_name = "java"

    def __init__(self, threads: int = 0, framework: str = "") -> None:
        self.threads = threads
        self.framework_override = framework
        self.project: Optional[ParsedProject] = None
        self._root: Optional[str] = None
        self._file_docs: Dict[str, dict] = {}

    # -- identity -------------------------------------------------------
    def language(self) -> str:
        return self.language_name

    def source_root(self) -> str:
        if self.project is not None:
            return self.project.source_root
        return self.default_source_root()

    def default_source_root(self) -> str:
        return "."

    # -- template method ------------------------------------------------
    def scan(self, project_root: str) -> ParsedProject:
        require_non_null(project_root, "Project root is required")
        t0 = time.perf_counter()
        doc = native_scan(project_root, self.language_name, self.threads, self.framework_override)
        self.project = to_parsed_project(doc)
        self._root = os.path.abspath(project_root)
        LOG.info("Scanned %s: %d files, %d units in %.1f ms (native %.1f ms)", project_root,
                 self.project.stats.get("analyzed", 0), len(self.project.units),
                 (time.perf_counter() - t0) * 1e3, self.project.stats.get("elapsedUs", 0) / 1e3)
        return self.project

    def scan_tree(self, tree, rows=None, isolate_timeout_s: Optional[float] = None) -> ParsedProject:
        """Scans a :class:`dmcp.index.source.SourceTree` (in-memory git snapshot
        or checkout) -- same result as :meth:`scan` over a checkout of it.
        ``rows``: :meth:`ProjectRowsWriter.static_rows` -- the native scan then
        hands the class / method rows to the writer before it builds any
        Python object (their ids in ``ParsedProject.static_row_ids``).
        ``isolate_timeout_s``: run the scan in a child process killed after
        that many seconds (:mod:`dmcp.parsers.isolated`: a persistent
        ``srcscan serve`` child whose binary result is decoded here, ``rows``
        honoured; a checkout directory goes to a one-shot JSON child).""" 
        t0 = time.perf_counter()
        timing: dict = {}
        if isolate_timeout_s:
            from . import isolated
            from ..index.source import CheckoutTree
            if isolated.objects_supported() and not isinstance(tree, CheckoutTree):
                # the persistent child: a binary result decoded natively, the
                # rows streamed to the writer as in process
                doc = isolated.scan_objects_in_child(tree, self.language_name, self.threads,
                                                     self.framework_override, isolate_timeout_s, rows=rows,
                                                     go_doc=rows is None, timing=timing)
            else:
                doc = isolated.scan_in_child(tree, self.language_name, self.threads, self.framework_override,
                                             isolate_timeout_s)
        else:
            doc = tree.scan_objects(self.language_name, self.threads, self.framework_override, rows=rows)
        if doc is None:
            doc = json.loads(tree.scan(self.language_name, self.threads, self.framework_override))
        t1 = time.perf_counter()
        self.project = to_parsed_project(doc)
        self.project.static_row_ids = doc.get("rowIds")
        self.project.scan_timing = dict(timing, objects_ms=(time.perf_counter() - t1) * 1e3)
        self._root = tree.directory
        LOG.info("Scanned %s @ %s: %d files, %d units in %.1f ms", tree.directory, tree.commit_hash[:12],
                 self.project.stats.get("analyzed", 0), len(self.project.units), (time.perf_counter() - t0) * 1e3)
        return self.project

    def parse(self, project_root: str) -> ProjectGraph:
        return self.scan(project_root).build_graph()

    # -- per-file hooks ----------------------------------------------------
    # Answered from the cached project scan when the file is part of it (the
    # indexing path); otherwise the file is analysed on its own by the native
    # front-end (``scan_file``), so the hooks also work stand-alone like the
    # reference's ``inferClassType(Path)`` / ``extractMethods(Path)`` /
    # ``extractMethodParameters(Path, Path, Set)`` (JavaSourceParser.java:236-436).
    def _unit_for(self, file_path: str) -> Optional[ParsedUnit]:
        if self.project is None:
            return None
        rel = file_path
        if self._root and os.path.isabs(file_path):
            rel = os.path.relpath(file_path, self._root)
        ident = self.project.file_to_identifier.get(rel.replace(os.sep, "/"))
        return self.project.units.get(ident) if ident else None

    def _file_doc(self, file_path: str) -> Optional[dict]:
        """Native single-file analysis (cached per path) for files outside the scan."""
        key = os.path.abspath(file_path)
        doc = self._file_docs.get(key)
        if doc is None:
            if not os.path.isfile(key):
                return None
            rel = os.path.relpath(key, self._root) if self._root else os.path.basename(key)
            doc = json.loads(native().scan_file(key, self.language_name, rel.replace(os.sep, "/"),
                                                self.framework_override))
            self._file_docs[key] = doc
        return doc if doc.get("parsed", True) else None

    def infer_class_type(self, file_path: str) -> ClassType:
        u = self._unit_for(file_path)
        if u is not None:
            return u.class_type
        doc = self._file_doc(file_path)
        return _class_type(doc.get("classType")) if doc else ClassType.OTHER

    def extract_methods(self, file_path: str) -> List[StaticMethodInfo]:
        u = self._unit_for(file_path)
        if u is not None:
            return list(u.methods)
        doc = self._file_doc(file_path)
        return _methods_from(doc.get("methods") or ()) if doc else []

    def extract_method_parameters(self, file_path: str, source_root: Optional[str] = None,
                                  known_identifiers: Optional[Set[str]] = None) -> Dict[str, List[str]]:
        """method name -> identifiers of its parameter types that are project
        classes (methods without any are omitted; the last overload wins)."""
        u = self._unit_for(file_path)
        if u is not None:
            if known_identifiers is None:
                return {k: list(v) for k, v in u.params.items()}
            return {k: [x for x in v if x in known_identifiers] for k, v in u.params.items()
                    if any(x in known_identifiers for x in v)}
        doc = self._file_doc(file_path)
        if not doc:
            return {}
        known = known_identifiers if known_identifiers is not None else set()
        resolve = self._param_resolver(doc, file_path, source_root, known)
        out: Dict[str, List[str]] = {}
        for rp in doc.get("rawParams") or ():
            if not rp.get("eligible", True):
                continue
            matched = [r for r in (resolve(t) for t in rp.get("types") or () if t) if r]
            if matched:
                out.pop(rp["name"], None)
                out[rp["name"]] = matched
        return out

    def _param_resolver(self, doc: dict, file_path: str, source_root: Optional[str], known: Set[str]):
        """Java ``resolveType`` (:505-530): known FQCN -> import map -> same package."""
        imports: Dict[str, str] = {}
        for imp in doc.get("imports") or ():
            if imp.get("isAsterisk"):
                continue
            fq = imp.get("importedName") or ""
            if imp.get("isStatic"):
                fq = fq.rsplit(".", 1)[0] if "." in fq else ""
            if "." in fq:
                imports[fq.rsplit(".", 1)[1]] = fq
        pkg = doc.get("package") or ""

        def resolve(ty: str) -> Optional[str]:
            if ty in known:
                return ty
            fq = imports.get(ty)
            if fq is not None and fq in known:
                return fq
            if pkg and f"{pkg}.{ty}" in known:
                return f"{pkg}.{ty}"
            return None
        return resolve

    def is_entry_point(self, file_path: str) -> bool:
        u = self._unit_for(file_path)
        if u is not None:
            return bool(u.entry_point)
        doc = self._file_doc(file_path)
        return bool(doc and doc.get("entryPoint"))


class JavaSourceParser(SourceParser):
    language_name = "java"

    def default_source_root(self) -> str:
        return "src/main/java"


class NodeJsSourceParser(SourceParser):
    """TypeScript / JavaScript (NodeJsGraalParser parity)."""

    language_name = "typescript"

    def default_source_root(self) -> str:
        return "src"

    def framework(self) -> Optional[dict]:
        return self.project.framework if self.project else None

    def _param_resolver(self, doc: dict, file_path: str, source_root: Optional[str], known: Set[str]):
        """NodeJsGraalParser ``extractMethodParameters`` / ``resolveImport``
        (:302-336, :371-401): a parameter type names an import's local binding;
        its relative module specifier resolves against the file's directory,
        inside ``source_root``, to ``a.b.c`` or ``a.b.c.index``."""
        root = os.path.abspath(source_root or os.path.join(self._root or os.path.dirname(file_path),
                                                           self.source_root()))
        here = os.path.dirname(os.path.abspath(file_path))
        locals_: Dict[str, str] = {}
        for imp in doc.get("imports") or ():
            spec = imp.get("source") or ""
            if not spec.startswith("."):
                continue
            full = os.path.normpath(os.path.join(here, spec))
            if not full.startswith(root + os.sep):
                continue
            cand = os.path.relpath(full, root).replace(os.sep, ".")
            for c in (cand, cand + ".index"):
                if c in known:
                    locals_[imp.get("localName") or ""] = c
                    break
        return locals_.get


class LegacyNodeJsSourceParser(NodeJsSourceParser):
    """The reference's unwired regex parser (``NodeJsSourceParser.java``,
    SURVEY §2.4 #33) as a mode of the same native front-end: its extra rules
    -- ``require('./x')`` dependencies, ``app.use(...)`` entry points -- are
    already production behaviour here; what differs is that it recognised
    NestJS ``@Get('/p')``-style verbs in any project (``:61-105, 304-377``),
    whereas the Babel path needs ``framework == nestjs``.  This mode keeps
    decorator routing on regardless of ``package.json``."""

    def __init__(self, threads: int = 0) -> None:
        super().__init__(threads, framework="nestjs")


class GoSourceParser(SourceParser):
    language_name = "go"

    def default_source_root(self) -> str:
        return "."

    def go_analysis(self) -> Optional[dict]:
        if self.project is None:
            return None
        go = self.project.go_analysis
        if isinstance(go, (str, bytes)):
            go = self.project.go_analysis = json.loads(go)
        return go


def parser_for(language: str, threads: int = 0) -> SourceParser:
    lang = (language or "java").lower()
    if lang in ("go", "golang"):
        return GoSourceParser(threads)
    if lang in ("typescript", "ts", "javascript", "js", "node", "nodejs"):
        return NodeJsSourceParser(threads)
    return JavaSourceParser(threads)


def detect_parser(root: str, threads: int = 0) -> SourceParser:
    return parser_for(detect_language(root), threads)


def unit_files(project: ParsedProject) -> Mapping[str, List[str]]:
    return {i: u.files for i, u in project.units.items()}
