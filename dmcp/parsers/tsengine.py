"""Per-file TS/JS analysis API over the native front-end.

Parity: ``analysis/domain/nodejs/GraalJsAnalyzerEngine.java`` (``detectFramework``
``:115-130``, ``analyzeFile`` ``:145-164``) and its DTOs ``FrameworkInfo``,
``RawImport``, ``MethodAnalysisResult``, ``FileAnalysisResult``
(``FrameworkInfo.java:17-21``, ``RawImport.java:17-21``,
``MethodAnalysisResult.java:19-25``, ``FileAnalysisResult.java:21-27``).

The reference loads a 1.7 MB Babel bundle into a GraalJS context and crosses
the polyglot boundary with JSON strings per file.  Here the same facts come
from the C++ front-end (``native/srcscan/ts_frontend.cpp``) in-process, with
the GIL released; an :class:`AnalyzerEngine` is stateless and cheap, so
``close()`` exists only for API parity.
"""
from __future__ import annotations

import json
from typing import Dict, List, NamedTuple, Optional, Tuple

from .base import native


class FrameworkInfo(NamedTuple):
    name: str
    source_root: str
    features: Dict[str, str]


class RawImport(NamedTuple):
    imported_name: str
    local_name: str
    source: str


class MethodAnalysisResult(NamedTuple):
    name: str
    line: int
    http_method: Optional[str]
    http_path: Optional[str]
    parameter_types: Tuple[str, ...]


class FileAnalysisResult(NamedTuple):
    path: str
    class_type: str
    entry_point: bool
    methods: Tuple[MethodAnalysisResult, ...]
    raw_imports: Tuple[RawImport, ...]


class AnalyzerEngine:
    """``GraalJsAnalyzerEngine`` equivalent (detect framework, analyse one file)."""

    def detect_framework(self, package_json: Optional[str]) -> FrameworkInfo:
        d = native().detect_framework(package_json or "{}")
        if isinstance(d, (bytes, str)):
            d = json.loads(d)
        return FrameworkInfo(d.get("name", "unknown"), d.get("sourceRoot", "src"), dict(d.get("features") or {}))

    def analyze_file(self, content: str, file_path: str, framework_name: Optional[str] = "unknown"
                     ) -> FileAnalysisResult:
        """Never raises on bad syntax: an unparsable file yields what could be
        recovered (typically nothing), like the Babel ``errorRecovery`` mode."""
        doc = json.loads(native().analyze_source(content or "", "typescript", file_path,
                                                 framework_name or "unknown"))
        # ``rawParams`` is emitted in method order, one entry per method
        raw = doc.get("rawParams") or ()
        methods: List[MethodAnalysisResult] = []
        for m, rp in zip(doc.get("methods") or (), raw):
            methods.append(MethodAnalysisResult(m["name"], m.get("line") or 0, m.get("httpMethod"),
                                                m.get("httpPath"), tuple(rp.get("types") or ())))
        imports = tuple(RawImport(i.get("importedName", ""), i.get("localName", ""), i.get("source", ""))
                        for i in doc.get("imports") or ())
        return FileAnalysisResult(doc.get("path", file_path), doc.get("classType") or "OTHER",
                                  bool(doc.get("entryPoint")), tuple(methods), imports)

    def close(self) -> None:
        pass

    def __enter__(self) -> "AnalyzerEngine":
        return self

    def __exit__(self, *exc) -> None:
        self.close()
