"""LLM response handling: JSON extraction, truncated-JSON repair, parsing.

Parity: ``ClaudeApiClient.java`` -- ``extractJson`` (``:576-603``: strip
markdown fences, slice the outermost ``{...}``), ``repairTruncatedJson``
(``:618-708``: cut at the last structurally complete ``}``/``]`` outside string
literals and append the missing closers), ``parseEnrichmentResponse``
(``:397-442``) and ``parseStringList`` (``:729-745``: a string or an array).
These were private and untested in the reference (SURVEY §4 gaps); here they
are public and unit-tested.
"""
from __future__ import annotations

import json
import logging
from typing import Any, List, Optional

from .types import EnrichmentResult, MethodEnrichment

LOG = logging.getLogger(__name__)


def extract_json(output: Optional[str]) -> str:
    if output is None or not output.strip():
        return "{}"
    cleaned = output.strip()
    if cleaned.startswith("```"):
        nl = cleaned.find("\n")
        if nl > 0:
            cleaned = cleaned[nl + 1:]
        if cleaned.endswith("```"):
            cleaned = cleaned[:cleaned.rfind("```")]
        cleaned = cleaned.strip()
    start = cleaned.find("{")
    end = cleaned.rfind("}")
    if start >= 0 and end > start:
        return cleaned[start:end + 1]
    return cleaned


def _scan(text: str):
    """Yields (index, char) for structural characters outside string literals and
    returns the final (braces, brackets, in_string) state via StopIteration value."""
    braces = brackets = 0
    in_string = escaped = False
    last_close = -1
    for i, c in enumerate(text):
        if escaped:
            escaped = False
            continue
        if c == "\\" and in_string:
            escaped = True
            continue
        if c == '"':
            in_string = not in_string
            continue
        if in_string:
            continue
        if c == "{":
            braces += 1
        elif c == "}":
            braces -= 1
            last_close = i
        elif c == "[":
            brackets += 1
        elif c == "]":
            brackets -= 1
            last_close = i
    return braces, brackets, in_string, last_close


def repair_truncated_json(text: str) -> str:
    braces, brackets, in_string, last_close = _scan(text)
    if braces == 0 and brackets == 0 and not in_string:
        return text
    truncated = text[:last_close + 1] if last_close > 0 else text
    # Close in proper nesting order (the reference appends all ']' then all '}').
    stack: List[str] = []
    in_str = esc = False
    for c in truncated:
        if esc:
            esc = False
            continue
        if c == "\\" and in_str:
            esc = True
            continue
        if c == '"':
            in_str = not in_str
            continue
        if in_str:
            continue
        if c in "{[":
            stack.append(c)
        elif c in "}]" and stack:
            stack.pop()
    repaired = truncated
    if in_str:
        repaired += '"'
    stripped = repaired.rstrip()
    if stripped.endswith(","):
        repaired = stripped[:-1]
    for opener in reversed(stack):
        repaired += "]" if opener == "[" else "}"
    return repaired


def parse_string_list(node: Any) -> List[str]:
    if node is None:
        return []
    if isinstance(node, str):
        t = node.strip()
        return [t] if t else []
    if isinstance(node, list):
        return [_as_text(x) for x in node]
    return []


def _as_text(x: Any) -> str:
    """Jackson ``JsonNode.asText`` semantics for array items."""
    if isinstance(x, str):
        return x
    if x is None:
        return "null"
    if isinstance(x, bool):
        return "true" if x else "false"
    if isinstance(x, (int, float)):
        return str(x)
    return ""  # containers have no text value


def _text_or(node: dict, key: str, default: Optional[str]) -> Optional[str]:
    v = node.get(key) if isinstance(node, dict) else None
    if v is None:
        return default
    if isinstance(v, str):
        return v
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, (int, float)):
        return str(v)
    return json.dumps(v)


def loads_lenient(raw: str) -> Any:
    """extract_json + json.loads, falling back to the truncation repair."""
    text = extract_json(raw)
    try:
        return json.loads(text)
    except ValueError as first:
        repaired = repair_truncated_json(text)
        try:
            value = json.loads(repaired)
        except ValueError:
            raise first
        LOG.warning("Repaired truncated JSON response; some entries may be missing")
        return value


def parse_enrichment_response(raw: Optional[str], full_class_name: str) -> EnrichmentResult:
    try:
        root = loads_lenient(raw or "")
    except ValueError as e:
        return EnrichmentResult.failure(full_class_name, f"JSON parse error: {e}")
    if not isinstance(root, dict):
        return EnrichmentResult.failure(full_class_name, "JSON parse error: top-level value is not an object")
    description = _text_or(root, "description", "")
    correction = _text_or(root, "classTypeCorrection", None)
    methods: List[MethodEnrichment] = []
    for m in root.get("methods") or []:
        if not isinstance(m, dict):
            continue
        methods.append(MethodEnrichment(_text_or(m, "methodName", "unknown"),
                                        _text_or(m, "description", ""),
                                        parse_string_list(m.get("businessLogic"))))
    return EnrichmentResult.ok(full_class_name, description, correction, methods)
