"""Enrichment backends: who writes the business descriptions.

Parity: ``analysis/domain/ClaudeApiClient.java`` -- enrichment prompt
(``:85-121``: source + statically inferred type + method names in, ``{description,
classTypeCorrection, methods[{methodName, description, businessLogic[]}]}``
out), ``enrichClass`` (``:288-329``; failures become failure results, never
exceptions) and ``enrichBatch`` (``:342-388``: one task per input, at most
``maxConcurrent`` in flight, results in input order).  The legacy
full-analysis path (``analyzeClass``/``analyzeBatch``, ``:164-275``) is dead
code in the reference and is provided as :meth:`AnthropicBackend.analyze_class`
for completeness.

Backends:

* :class:`AnthropicBackend` -- Messages API over HTTPS (stdlib ``urllib``),
  model/max-tokens/timeout/retries from config (the reference hard-codes them).
* :class:`NullBackend`      -- enrichment disabled (static indexing only).
* :class:`FakeBackend`      -- deterministic, offline; used by tests and benches.
* ``LocalLLMBackend``       -- optional MI355X extension (:mod:`dmcp.enrich.local`).
"""
from __future__ import annotations

import json
import logging
import os
import random
import threading
import time
import urllib.error
import urllib.request
from concurrent.futures import FIRST_COMPLETED, Future, ThreadPoolExecutor, wait
from typing import Callable, Dict, Iterable, Iterator, List, Optional, Sequence, Tuple

from ..utils.errors import require_non_blank, require_non_null
from .jsonfix import parse_enrichment_response
from .types import (BatchClassInput, ClassAnalysisResult, EnrichmentInput, EnrichmentResult,
                    MethodAnalysisResult)

LOG = logging.getLogger(__name__)

# The per-project part (task, reply schema, rules, README) comes first and
# everything per class after "Source of": a local engine prefills that part
# once per project and reads it through the shared-prefix attention, so each
# class costs only its own source and facts (dmcp/enrich/local.py).
ENRICHMENT_PROMPT = """\
You are adding business context to the source files of one project that have already
been parsed statically, one file per request.

Describe what the code means for the business, not how it is implemented.
Answer with exactly one JSON object of this shape and nothing else:
{{
  "description": "one sentence on the business purpose of this class/module",
  "classTypeCorrection": "a corrected class type, or null when the extracted class type is right",
  "methods": [
    {{"methodName": "a method name from the extracted method list",
      "description": "one sentence of business meaning",
      "businessLogic": ["business step 1", "business step 2"]}}
  ]
}}
Rules: cover every listed method; change the class type only when it is clearly wrong
(valid types: CONTROLLER, SERVICE, REPOSITORY, ENTITY, DTO, CONFIGURATION, LISTENER,
UTILITY, EXCEPTION, OTHER); the first character of the reply must be {{ and the last }}.

Project context (README):
{readme}

Source of {name}:
```{language}
{source}
```

Statically extracted facts:
- Class type: {class_type}
- Methods: {methods}

The JSON object for {name}:
"""

ANALYSIS_PROMPT = """\
You are analyzing one {language} source file of a project.

Project context (README):
{readme}

Source of {name}:
```{language}
{source}
```

Reply with one JSON object: {{"fullClassName", "classType", "description", "sourceFile",
"methods": [{{"methodName", "description", "businessLogic": [], "exceptions": [],
"httpMethod", "httpPath", "lineNumber"}}]}}. Describe business meaning, include every
public method, one sentence per description, and output raw JSON only.
"""


def build_enrichment_prompt(inp: EnrichmentInput, readme: Optional[str],
                            max_source_chars: int = 0) -> str:
    src = inp.source_code
    if max_source_chars and len(src) > max_source_chars:
        src = src[:max_source_chars] + "\n...(truncated)"
    return ENRICHMENT_PROMPT.format(
        language=inp.language or "java",
        readme=readme if readme and readme.strip() else "No README available.",
        name=inp.full_class_name, source=src, class_type=inp.class_type,
        methods=", ".join(inp.method_names))


# enrichment_source values (source_classes.enrichment_source) of backends
# whose descriptions carry no information about the code: random-initialised
# local presets, the model-free echo engine, the offline fake.  Phase 3 and
# resume-enrichment redo such rows once a real backend is configured.
SYNTHETIC_PREFIX = "synthetic:"


def is_synthetic(source_tag: Optional[str]) -> bool:
    return bool(source_tag) and source_tag.startswith(SYNTHETIC_PREFIX)


class EnrichmentBackend:
    """Base: subclasses implement :meth:`enrich_class`; the batch fan-out is shared."""

    name = "base"

    @property
    def source_tag(self) -> str:
        """What the enrichment rows written through this backend record as
        their ``enrichment_source`` (:data:`SYNTHETIC_PREFIX`: placeholder
        descriptions a real backend replaces)."""
        return self.name

    def __init__(self, max_concurrent: int = 5) -> None:
        self.max_concurrent = max(1, int(max_concurrent))
        self._pool: Optional[ThreadPoolExecutor] = None
        self._pool_lock = threading.Lock()

    @property
    def enabled(self) -> bool:
        return True

    def enrich_class(self, inp: EnrichmentInput, readme: Optional[str]) -> EnrichmentResult:
        raise NotImplementedError

    def _executor(self) -> ThreadPoolExecutor:
        with self._pool_lock:
            if self._pool is None:
                self._pool = ThreadPoolExecutor(max_workers=self.max_concurrent,
                                                thread_name_prefix=f"enrich-{self.name}")
            return self._pool

    def _safe(self, inp: EnrichmentInput, readme: Optional[str]) -> EnrichmentResult:
        try:
            return self.enrich_class(inp, readme)
        except Exception as e:  # isolate per-class failures (ClaudeApiClient.java:322-328)
            LOG.warning("Enrichment failed for %s: %s", inp.full_class_name, e)
            return EnrichmentResult.failure(inp.full_class_name, str(e))

    def enrich_batch(self, inputs: Sequence[EnrichmentInput], readme: Optional[str]) -> List[EnrichmentResult]:
        require_non_null(inputs, "Inputs list is required")
        if not inputs:
            return []
        if self.max_concurrent == 1 or len(inputs) == 1:
            return [self._safe(i, readme) for i in inputs]
        ex = self._executor()
        futures = [ex.submit(self._safe, i, readme) for i in inputs]
        out = []
        for inp, fut in zip(inputs, futures):
            try:
                out.append(fut.result())
            except Exception as e:
                out.append(EnrichmentResult.failure(inp.full_class_name, str(e)))
        return out

    def enrich_stream(self, inputs: Iterable[EnrichmentInput], readme: Optional[str]
                      ) -> Iterator[Tuple[int, EnrichmentResult]]:
        """Yields ``(input index, result)`` in completion order, with at most
        ``max_concurrent`` classes in flight and the next one submitted as
        soon as one finishes (a sliding window instead of the reference's
        barrier per batch of 20, ``CodeContextService.java:297-359``, which
        waits for the slowest of every 20).  ``inputs`` is consumed lazily."""
        it = enumerate(inputs)
        if self.max_concurrent == 1:
            for i, inp in it:
                yield i, self._safe(inp, readme)
            return
        ex = self._executor()
        live: Dict[Future, Tuple[int, EnrichmentInput]] = {}
        exhausted = False
        while True:
            while not exhausted and len(live) < self.max_concurrent:
                try:
                    i, inp = next(it)
                except StopIteration:
                    exhausted = True
                    break
                live[ex.submit(self._safe, inp, readme)] = (i, inp)
            if not live:
                return
            done, _ = wait(list(live), return_when=FIRST_COMPLETED)
            for f in done:
                i, inp = live.pop(f)
                try:
                    yield i, f.result()
                except Exception as e:
                    yield i, EnrichmentResult.failure(inp.full_class_name, str(e))

    def close(self) -> None:
        with self._pool_lock:
            if self._pool is not None:
                self._pool.shutdown(wait=False)
                self._pool = None


class NullBackend(EnrichmentBackend):
    name = "null"

    @property
    def enabled(self) -> bool:
        return False

    def enrich_class(self, inp: EnrichmentInput, readme: Optional[str]) -> EnrichmentResult:
        return EnrichmentResult.failure(inp.full_class_name, "enrichment disabled")


class RefusedBackend(NullBackend):
    """A configured backend that must not run: analysis then refuses like the
    reference's READ_ONLY_MODE (``CodeContextService.java:149-156``) with
    :attr:`disabled_reason` as the message, or indexes statically when
    ``REQUIRE_ENRICHMENT_FOR_ANALYZE=false``."""

    name = "refused"

    def __init__(self, reason: str) -> None:
        super().__init__(1)
        self.disabled_reason = reason

    def enrich_class(self, inp: EnrichmentInput, readme: Optional[str]) -> EnrichmentResult:
        return EnrichmentResult.failure(inp.full_class_name, self.disabled_reason)


class FakeBackend(EnrichmentBackend):
    """Deterministic offline backend.

    ``responder`` (optional) maps an input to raw model text, which then goes
    through the same JSON extraction/repair path as a real reply -- tests use
    it to inject fenced, truncated or malformed replies and failures.
    """

    name = "fake"
    source_tag = SYNTHETIC_PREFIX + "fake"

    def __init__(self, max_concurrent: int = 5,
                 responder: Optional[Callable[[EnrichmentInput], str]] = None,
                 latency_s: float = 0.0) -> None:
        super().__init__(max_concurrent)
        self.responder = responder
        self.latency_s = latency_s
        self.calls: List[str] = []
        self._lock = threading.Lock()

    def enrich_class(self, inp: EnrichmentInput, readme: Optional[str]) -> EnrichmentResult:
        with self._lock:
            self.calls.append(inp.full_class_name)
        if self.latency_s:
            time.sleep(self.latency_s)
        if self.responder is not None:
            return parse_enrichment_response(self.responder(inp), inp.full_class_name)
        simple = inp.full_class_name.rsplit(".", 1)[-1]
        reply = {
            "description": f"{simple} handles the {simple.lower()} business capability",
            "classTypeCorrection": None,
            "methods": [{"methodName": m, "description": f"Performs {m}",
                         "businessLogic": [f"Validate {m} input", f"Apply {m} rule"]}
                        for m in inp.method_names],
        }
        return parse_enrichment_response(json.dumps(reply), inp.full_class_name)


class AnthropicBackend(EnrichmentBackend):
    """Anthropic Messages API client (stdlib HTTP, retries with backoff)."""

    name = "anthropic"

    @property
    def source_tag(self) -> str:
        return f"anthropic:{self.model}"
    API_VERSION = "2023-06-01"

    def __init__(self, api_key: str, model: str, max_tokens: int = 16384, timeout_s: float = 240.0,
                 max_retries: int = 2, max_concurrent: int = 5,
                 base_url: str = "https://api.anthropic.com", max_source_chars: int = 0) -> None:
        super().__init__(max_concurrent)
        self.api_key = require_non_blank(api_key, "API key is required")
        self.model = model
        self.max_tokens = int(max_tokens)
        self.timeout_s = float(timeout_s)
        self.max_retries = int(max_retries)
        self.base_url = base_url.rstrip("/")
        self.max_source_chars = max_source_chars

    def _post(self, prompt: str) -> str:
        body = json.dumps({"model": self.model, "max_tokens": self.max_tokens,
                           "messages": [{"role": "user", "content": prompt}]}).encode("utf-8")
        req = urllib.request.Request(f"{self.base_url}/v1/messages", data=body, method="POST", headers={
            "content-type": "application/json", "x-api-key": self.api_key,
            "anthropic-version": self.API_VERSION})
        attempt = 0
        while True:
            try:
                with urllib.request.urlopen(req, timeout=self.timeout_s) as resp:
                    payload = json.loads(resp.read().decode("utf-8"))
                return "".join(block.get("text", "") for block in payload.get("content", [])
                               if block.get("type") == "text")
            except urllib.error.HTTPError as e:
                retryable = e.code in (408, 409, 429) or e.code >= 500
                if not retryable or attempt >= self.max_retries:
                    detail = e.read().decode("utf-8", "replace")[:500] if hasattr(e, "read") else ""
                    raise RuntimeError(f"HTTP {e.code}: {detail}") from e
            except (urllib.error.URLError, TimeoutError, ConnectionError) as e:
                if attempt >= self.max_retries:
                    raise RuntimeError(f"request failed: {e}") from e
            attempt += 1
            time.sleep(min(8.0, 0.5 * 2 ** attempt) * (0.75 + random.random() / 2))

    def enrich_class(self, inp: EnrichmentInput, readme: Optional[str]) -> EnrichmentResult:
        require_non_null(inp, "Enrichment input is required")
        raw = self._post(build_enrichment_prompt(inp, readme, self.max_source_chars))
        return parse_enrichment_response(raw, inp.full_class_name)

    def analyze_class(self, source_code: str, full_class_name: str, source_file: Optional[str],
                      readme: Optional[str], language: Optional[str]) -> ClassAnalysisResult:
        """Legacy single-shot analysis (``analyzeClass`` :164-209, dead code in
        the reference): arguments are validated eagerly, a failed call or an
        unparsable reply becomes a failure result."""
        require_non_blank(source_code, "Source code is required")
        require_non_blank(full_class_name, "Full class name is required")
        prompt = ANALYSIS_PROMPT.format(language=language or "java",
                                        readme=readme or "No README available.",
                                        name=full_class_name, source=source_code)
        try:
            return parse_analysis_response(self._post(prompt), full_class_name, source_file)
        except Exception as e:
            LOG.warning("Analysis failed for %s: %s", full_class_name, e)
            return ClassAnalysisResult.failure(full_class_name, source_file, str(e))

    def analyze_batch(self, inputs: Sequence[BatchClassInput], readme: Optional[str]
                      ) -> List[ClassAnalysisResult]:
        """``analyzeBatch`` (:223-275): one task per input, bounded fan-out,
        results in input order, per-input failure isolation."""
        require_non_null(inputs, "Inputs list is required")
        if not inputs:
            return []

        def one(i: BatchClassInput) -> ClassAnalysisResult:
            try:
                return self.analyze_class(i.source_code, i.full_class_name, i.source_file, readme, i.language)
            except Exception as e:
                return ClassAnalysisResult.failure(i.full_class_name, i.source_file, str(e))
        return list(self._executor().map(one, inputs))


def parse_analysis_response(raw: str, full_class_name: str, source_file: Optional[str]) -> ClassAnalysisResult:
    """Legacy reply ``{fullClassName, classType, description, sourceFile, methods[]}``."""
    from .jsonfix import loads_lenient, parse_string_list
    root = loads_lenient(raw)
    if not isinstance(root, dict):
        return ClassAnalysisResult.failure(full_class_name, source_file, "reply is not a JSON object")
    methods = []
    for m in root.get("methods") or ():
        if not isinstance(m, dict) or not m.get("methodName"):
            continue
        ln = m.get("lineNumber")
        methods.append(MethodAnalysisResult(
            str(m["methodName"]), m.get("description"), parse_string_list(m.get("businessLogic")),
            parse_string_list(m.get("exceptions")), m.get("httpMethod") or None, m.get("httpPath") or None,
            int(ln) if isinstance(ln, (int, float)) else None))
    return ClassAnalysisResult.ok(str(root.get("fullClassName") or full_class_name),
                                  str(root.get("classType") or "OTHER"), root.get("description"),
                                  root.get("sourceFile") or source_file, methods)


class LazyBackend(EnrichmentBackend):
    """A backend built on its first enrichment call.

    The local MI355X backend spawns one worker process per GPU and each
    allocates a KV-cache slab of tens of GB; a process that never enriches
    -- the read-only MCP server (``application-mcp.yml:1-8``: no web stack,
    only the 9 query tools), a REST instance that only answers queries --
    must not pay for it.  ``enabled`` is known without building (analysis
    mode checks it, ``CodeContextService.java:149-156``)."""

    def __init__(self, factory: Callable[[], EnrichmentBackend], name: str = "lazy",
                 enabled: bool = True, source_tag: Optional[str] = None) -> None:
        super().__init__(1)
        self._factory = factory
        self._enabled = enabled
        self._source_tag = source_tag
        self._built: Optional[EnrichmentBackend] = None
        self._build_lock = threading.Lock()
        self.name = name

    @property
    def enabled(self) -> bool:
        return self._enabled

    @property
    def built(self) -> bool:
        return self._built is not None

    @property
    def source_tag(self) -> str:  # known without building (the rows' tag)
        if self._source_tag is not None:
            return self._source_tag
        return self.get().source_tag

    def get(self) -> EnrichmentBackend:
        with self._build_lock:
            if self._built is None:
                LOG.info("Starting the %s enrichment backend", self.name)
                self._built = self._factory()
            return self._built

    def enrich_class(self, inp: EnrichmentInput, readme: Optional[str]) -> EnrichmentResult:
        return self.get().enrich_class(inp, readme)

    def enrich_batch(self, inputs: Sequence[EnrichmentInput], readme: Optional[str]) -> List[EnrichmentResult]:
        return self.get().enrich_batch(inputs, readme)

    def enrich_stream(self, inputs: Iterable[EnrichmentInput], readme: Optional[str]
                      ) -> Iterator[Tuple[int, EnrichmentResult]]:
        return self.get().enrich_stream(inputs, readme)

    def stats(self) -> dict:
        b = self._built
        return b.stats() if b is not None and hasattr(b, "stats") else {}

    def close(self) -> None:
        with self._build_lock:
            if self._built is not None:
                self._built.close()
        super().close()


def create_backend(cfg) -> EnrichmentBackend:
    """Backend selection from :class:`dmcp.config.Config`."""
    kind = cfg.resolved_enrich_backend()
    if kind == "anthropic":
        return AnthropicBackend(cfg.anthropic_api_key or "", cfg.claude_model, cfg.claude_max_tokens,
                                cfg.claude_timeout_seconds, cfg.claude_max_retries,
                                cfg.enrich_max_concurrent, cfg.anthropic_base_url,
                                cfg.enrich_max_source_chars)
    if kind == "fake":
        return FakeBackend(cfg.enrich_max_concurrent)
    if kind == "local":
        tag = local_source_tag(cfg)
        if is_synthetic(tag) and not getattr(cfg, "local_llm_allow_random_weights", False):
            reason = (f"ENRICH_BACKEND=local has no checkpoint (LOCAL_LLM_MODEL_PATH is unset): the "
                      f"{cfg.local_llm_preset!r} preset's random-initialised weights would write noise "
                      f"descriptions. Set LOCAL_LLM_MODEL_PATH to a Llama-format checkpoint directory, or "
                      f"LOCAL_LLM_ALLOW_RANDOM_WEIGHTS=true for benchmarks and tests")
            LOG.error("%s", reason)
            return RefusedBackend(reason)

        def build() -> EnrichmentBackend:
            from .local import LocalLLMBackend
            return LocalLLMBackend.from_config(cfg)
        return LazyBackend(build, "local", source_tag=tag)
    return NullBackend(1)


def local_source_tag(cfg) -> str:
    """``enrichment_source`` of the local backend: the checkpoint directory,
    or a synthetic tag for the random-initialised presets and the echo
    engine."""
    path = (getattr(cfg, "local_llm_model_path", "") or "").strip()
    if path:
        return f"local:{os.path.abspath(path)}"
    preset = getattr(cfg, "local_llm_preset", "") or "dmcp-coder-1b"
    return SYNTHETIC_PREFIX + ("echo" if preset == "echo" else f"random-init:{preset}")
