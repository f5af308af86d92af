"""Enrichment DTOs (``ClaudeApiClient.java:453-513``)."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional


@dataclass(frozen=True)
class EnrichmentInput:
    source_code: str
    full_class_name: str
    language: str
    class_type: str
    method_names: List[str] = field(default_factory=list)


@dataclass(frozen=True)
class MethodEnrichment:
    method_name: str
    description: str
    business_logic: List[str] = field(default_factory=list)


@dataclass(frozen=True)
class EnrichmentResult:
    success: bool
    full_class_name: str
    description: Optional[str] = None
    class_type_correction: Optional[str] = None
    methods: List[MethodEnrichment] = field(default_factory=list)
    error_message: Optional[str] = None

    @classmethod
    def ok(cls, full_class_name: str, description: str, class_type_correction: Optional[str],
           methods: List[MethodEnrichment]) -> "EnrichmentResult":
        return cls(True, full_class_name, description, class_type_correction, list(methods), None)

    @classmethod
    def failure(cls, full_class_name: str, error_message: Optional[str]) -> "EnrichmentResult":
        return cls(False, full_class_name, None, None, [], error_message)


def normalize_method_name(name: Optional[str]) -> Optional[str]:
    """Strips an LLM-added parenthetical qualifier: ``"onSuccess (loginMutation)"``
    -> ``"onSuccess"`` (CodeContextService.java:713-722)."""
    if name is None:
        return None
    i = name.find("(")
    if i > 0:
        return name[:i].strip()
    return name.strip()


# -- legacy full-analysis DTOs (ClaudeApiClient.java:453-513, 750-810) --------
@dataclass(frozen=True)
class MethodAnalysisResult:
    method_name: str
    description: Optional[str]
    business_logic: List[str] = field(default_factory=list)
    exceptions: List[str] = field(default_factory=list)
    http_method: Optional[str] = None
    http_path: Optional[str] = None
    line_number: Optional[int] = None


@dataclass(frozen=True)
class ClassAnalysisResult:
    success: bool
    full_class_name: str
    class_type: str
    description: Optional[str]
    source_file: Optional[str]
    methods: List[MethodAnalysisResult] = field(default_factory=list)
    error_message: Optional[str] = None

    @classmethod
    def ok(cls, full_class_name: str, class_type: str, description: Optional[str],
           source_file: Optional[str], methods: List[MethodAnalysisResult]) -> "ClassAnalysisResult":
        return cls(True, full_class_name, class_type, description, source_file, list(methods or []), None)

    @classmethod
    def failure(cls, full_class_name: str, source_file: Optional[str],
                error_message: Optional[str]) -> "ClassAnalysisResult":
        return cls(False, full_class_name, "OTHER", None, source_file, [], error_message)


@dataclass(frozen=True)
class BatchClassInput:
    source_code: str
    full_class_name: str
    source_file: str
    language: str


class SizedIter:
    """A lazy iterable that knows how many items it will (at most) yield:
    ``operator.length_hint`` reports ``n``, so a backend can deal the
    pending work evenly without materialising it."""

    def __init__(self, it, n: int) -> None:
        self._it = it
        self._n = int(n)

    def __length_hint__(self) -> int:
        return self._n

    def __iter__(self):
        return iter(self._it)
