"""Typed view of the Go analyzer's JSON contract.

Parity: ``analysis/domain/golang/GoAnalysisResult.java:21-168`` (Jackson
records with ``ignoreUnknown``) mirroring ``tools/go-analyzer/pkg/analysis/
types.go:10-175``.  The native Go front-end (``native/srcscan/go_frontend.cpp``,
``dmcp._srcscan.analyze_go``) emits exactly this document; :func:`analyze_go`
returns it as immutable records.  Unknown keys are ignored and missing or
``null`` collections become empty tuples, as the Java mapping does.
"""
from __future__ import annotations

import json
from typing import Any, Mapping, NamedTuple, Optional, Tuple, Union

from .base import native


def _s(d: Mapping[str, Any], k: str) -> str:
    v = d.get(k)
    return "" if v is None else str(v)


def _strs(d: Mapping[str, Any], k: str) -> Tuple[str, ...]:
    return tuple(str(x) for x in d.get(k) or ())


class GoParamInfo(NamedTuple):
    name: str
    type_name: str
    package_path: str
    is_pointer: bool
    is_slice: bool
    is_variadic: bool

    @classmethod
    def from_dict(cls, d: Mapping[str, Any]) -> "GoParamInfo":
        return cls(_s(d, "name"), _s(d, "type"), _s(d, "package"), bool(d.get("isPointer")),
                   bool(d.get("isSlice")), bool(d.get("isVariadic")))


class GoFieldInfo(NamedTuple):
    name: str
    type_name: str
    package_path: str
    is_exported: bool
    tag: str

    @classmethod
    def from_dict(cls, d: Mapping[str, Any]) -> "GoFieldInfo":
        return cls(_s(d, "name"), _s(d, "type"), _s(d, "package"), bool(d.get("isExported")), _s(d, "tag"))


class GoFunctionInfo(NamedTuple):
    name: str
    file: str
    line: int
    receiver: str
    params: Tuple[GoParamInfo, ...]
    returns: Tuple[str, ...]
    http_method: str
    http_path: str
    has_panic: bool
    doc: str

    @classmethod
    def from_dict(cls, d: Mapping[str, Any]) -> "GoFunctionInfo":
        return cls(_s(d, "name"), _s(d, "file"), int(d.get("line") or 0), _s(d, "receiver"),
                   tuple(GoParamInfo.from_dict(p) for p in d.get("params") or ()), _strs(d, "returns"),
                   _s(d, "httpMethod"), _s(d, "httpPath"), bool(d.get("hasPanic")), _s(d, "doc"))


class GoStructInfo(NamedTuple):
    name: str
    file: str
    line: int
    fields: Tuple[GoFieldInfo, ...]
    methods: Tuple[GoFunctionInfo, ...]
    embedded_types: Tuple[str, ...]
    implements: Tuple[str, ...]

    @classmethod
    def from_dict(cls, d: Mapping[str, Any]) -> "GoStructInfo":
        return cls(_s(d, "name"), _s(d, "file"), int(d.get("line") or 0),
                   tuple(GoFieldInfo.from_dict(f) for f in d.get("fields") or ()),
                   tuple(GoFunctionInfo.from_dict(m) for m in d.get("methods") or ()),
                   _strs(d, "embeddedTypes"), _strs(d, "implements"))


class GoMethodSignature(NamedTuple):
    name: str
    params: Tuple[GoParamInfo, ...]
    returns: Tuple[str, ...]

    @classmethod
    def from_dict(cls, d: Mapping[str, Any]) -> "GoMethodSignature":
        return cls(_s(d, "name"), tuple(GoParamInfo.from_dict(p) for p in d.get("params") or ()),
                   _strs(d, "returns"))


class GoInterfaceInfo(NamedTuple):
    name: str
    file: str
    line: int
    methods: Tuple[GoMethodSignature, ...]
    embedded_interfaces: Tuple[str, ...]

    @classmethod
    def from_dict(cls, d: Mapping[str, Any]) -> "GoInterfaceInfo":
        return cls(_s(d, "name"), _s(d, "file"), int(d.get("line") or 0),
                   tuple(GoMethodSignature.from_dict(m) for m in d.get("methods") or ()),
                   _strs(d, "embeddedInterfaces"))


class GoPackageInfo(NamedTuple):
    path: str
    name: str
    dir: str
    files: Tuple[str, ...]
    imports: Tuple[str, ...]
    structs: Tuple[GoStructInfo, ...]
    interfaces: Tuple[GoInterfaceInfo, ...]
    functions: Tuple[GoFunctionInfo, ...]
    is_entry_point: bool
    class_type: str

    @classmethod
    def from_dict(cls, d: Mapping[str, Any]) -> "GoPackageInfo":
        return cls(_s(d, "path"), _s(d, "name"), _s(d, "dir"), _strs(d, "files"), _strs(d, "imports"),
                   tuple(GoStructInfo.from_dict(s) for s in d.get("structs") or ()),
                   tuple(GoInterfaceInfo.from_dict(i) for i in d.get("interfaces") or ()),
                   tuple(GoFunctionInfo.from_dict(f) for f in d.get("functions") or ()),
                   bool(d.get("isEntryPoint")), _s(d, "classType") or "OTHER")


class GoAnalysisResult(NamedTuple):
    module: str
    packages: Tuple[GoPackageInfo, ...]

    @classmethod
    def from_dict(cls, d: Mapping[str, Any]) -> "GoAnalysisResult":
        return cls(_s(d, "module"), tuple(GoPackageInfo.from_dict(p) for p in d.get("packages") or ()))

    @classmethod
    def from_json(cls, text: Union[str, bytes]) -> "GoAnalysisResult":
        return cls.from_dict(json.loads(text))

    def package(self, path: str) -> Optional[GoPackageInfo]:
        return next((p for p in self.packages if p.path == path), None)


def analyze_go(project_root: str, threads: int = 0) -> GoAnalysisResult:
    """``go-analyzer <root>`` equivalent, in-process (no subprocess, no Go toolchain)."""
    return GoAnalysisResult.from_json(native().analyze_go(project_root, int(threads)))
