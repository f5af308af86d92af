"""Local enrichment backend on MI355X: a continuous-batching, JSON-constrained
generation engine over :class:`dmcp.models.llm.LocalLM` -- extension.

The reference sends every class to the Anthropic API, 5 requests at a time
(``ClaudeApiClient.java:342-388``); enrichment wall-clock dominates its
pipeline (SURVEY §3.2 hot loop #3).  This backend keeps the same contract
(:class:`EnrichmentInput` in, :class:`EnrichmentResult` out, failures isolated
per class) but generates on the local GPU:

* **schema-constrained decoding** -- the reply's JSON skeleton
  (``{"description": "...", "classTypeCorrection": null, "methods": [...]}``
  with every extracted method name) is *forced*; only string contents are
  generated, with a masked greedy argmax restricted to JSON-safe printable
  characters.  The output always parses, so Phase 3 recovery is only needed
  for infrastructure failures;
* **continuous batching** -- up to ``max_batch`` sequences decode together;
  finished sequences free their KV slot for the next prompt;
* **jump-forward** -- forced skeleton bytes are appended as extra rows of the
  same batched step (an exact multi-token extend), so only sampled tokens
  cost a step;
* each step is one H2D copy, one hipGraph replay (:class:`DecodeGraphs`:
  forward + gfx950 masked argmax with a per-row grammar-mask index) and one
  small D2H copy of the selected ids;
* **one-step pipeline** -- step t+1 is launched before step t's ids reach
  the host: a row whose token is step t's selection names its source row and
  the graph gathers it on the device; the host runs the grammar state machine
  for step t while the GPU computes step t+1, so host bookkeeping (~0.3 ms
  per step) leaves the critical path;
* streaming: :meth:`LocalEngine.stream` pulls classes from a feed as KV
  slots free up and yields each reply as soon as it is complete, so the
  indexing pipeline hands it ALL pending classes at once (no 20-class
  barriers) and applies results while the GPU keeps decoding;
* batched prefill: every class admitted in a step is prefilled in one pass
  (:meth:`LocalLM.prefill_batch`: one GEMM per projection over all their
  tokens, one variable-length attention launch);
* multi-GPU: one engine per GPU in its own worker process
  (:mod:`dmcp.enrich.workers`), all pulling from one queue -- pure data
  parallelism, no collectives.
"""
from __future__ import annotations

import gc
import json
import logging
import os
import threading
import time
from collections import deque
from dataclasses import dataclass, field
from typing import Any, Deque, Dict, Iterable, Iterator, List, Optional, Sequence, Tuple

import torch

from ..models.llm import LocalLM, LMConfig, DecodeGraphs, preset
from .backend import SYNTHETIC_PREFIX, EnrichmentBackend, build_enrichment_prompt
from .jsonfix import parse_enrichment_response
from .tokenizer import ByteTokenizer
from .tokenizer import _Base as _TokBase
from .types import EnrichmentInput, EnrichmentResult

LOG = logging.getLogger(__name__)

QUOTE = ord('"')


def _json_safe_mask(vocab: int, with_quote: bool) -> List[int]:
    """The byte vocabulary's free-text mask (tests; engines use the tokenizer's)."""
    words = [0] * ((vocab + 31) // 32)
    for b in range(0x20, 0x7F):
        if b in (QUOTE, ord("\\")):
            continue
        words[b >> 5] |= 1 << (b & 31)
    if with_quote:
        words[QUOTE >> 5] |= 1 << (QUOTE & 31)
    # int32 view of the uint32 bit pattern
    return [w - (1 << 32) if w >= (1 << 31) else w for w in words]

# The reference's reply contract (ClaudeApiClient.java:101-120): the model may
# correct the statically inferred class type (null = keep it; applied at
# CodeContextService.java:635-637) and writes 1..N business-logic steps per
# method.  Both are grammar CHOICES here: the model picks among the
# alternatives' bytes under per-state vocabulary masks.
CLASS_TYPES = ("CONTROLLER", "SERVICE", "REPOSITORY", "ENTITY", "DTO", "CONFIGURATION", "LISTENER", "UTILITY",
               "EXCEPTION", "OTHER")
CHOICE_CLASS_TYPE = 0   # null, or one of the 10 ClassType names (quoted)
CHOICE_MORE_STEPS = 1   # after a businessLogic step: "]" closes the list, ', "' opens another step
CHOICES: Dict[int, Tuple[bytes, ...]] = {
    CHOICE_CLASS_TYPE: (b"null",) + tuple(b'"' + t.encode() + b'"' for t in CLASS_TYPES),
    CHOICE_MORE_STEPS: (b"]", b', "'),
}


@dataclass
class Segment:
    """One piece of a reply: ``forced`` bytes, a free JSON string closed by
    the lone quote token -- at least ``min_len`` sampled tokens, at most
    ``max_len`` bytes (a length in text, whatever the tokenizer: a 4-byte
    BPE piece fills it 4x faster than a byte token) -- or a
    ``choice`` among :data:`CHOICES` alternatives (``then[k]``: the segments
    that follow alternative k)."""
    forced: Optional[bytes] = None
    min_len: int = 0
    max_len: int = 0
    ids: Optional[List[int]] = None  # the forced bytes as tokens (set by the engine's tokenizer)
    choice: int = -1
    then: Optional[List[List["Segment"]]] = None

    @property
    def is_free(self) -> bool:
        return self.forced is None and self.choice < 0


def _merge(segs: List[Segment]) -> List[Segment]:
    out: List[Segment] = []
    for s in segs:
        if out and s.forced is not None and out[-1].forced is not None:
            out[-1] = Segment(out[-1].forced + s.forced)
        else:
            out.append(s)
    return out


def _steps_chain(step_len: Tuple[int, int], max_steps: int, depth: int = 1) -> List[Segment]:
    """Business-logic step ``depth`` (its opening quote already emitted) and,
    below ``max_steps``, the model's choice to stop or open the next one."""
    segs = [Segment(None, *step_len)]
    if depth < max_steps:
        segs.append(Segment(choice=CHOICE_MORE_STEPS,
                            then=[[], _merge(_steps_chain(step_len, max_steps, depth + 1))]))
    else:
        segs.append(Segment(b"]"))
    return segs


@dataclass(frozen=True)
class ReplyShape:
    """Byte caps of the reply's free strings and the business-logic step
    count: the class description, each method's description, each step.
    The reference asks for a free business-oriented description, a
    1-sentence description per method and a list of steps under a
    16,384-token ``max_tokens`` (``ClaudeApiClient.java:40, 101-113``);
    :meth:`from_budget` derives the caps from the engine's reply budget
    (config ``LOCAL_LLM_DESC_MAX_BYTES`` / ``LOCAL_LLM_METHOD_MAX_BYTES`` /
    ``LOCAL_LLM_STEP_MAX_BYTES`` / ``LOCAL_LLM_MAX_STEPS`` override each;
    0 = derived).  :func:`plan_reply` / :func:`plan_branches` still shrink
    them for a class whose methods would not fit the budget."""
    desc: int = 96
    method: int = 64
    step: int = 40
    max_steps: int = 3

    LEGACY = None  # set below: the round-4 fixed caps (96 / 64 / 40 bytes, 3 steps)

    @classmethod
    def from_budget(cls, budget: int, desc: int = 0, method: int = 0, step: int = 0,
                    max_steps: int = 0) -> "ReplyShape":
        """Defaults scale with the reply budget (tokens): 1/16 of it for the
        class description (96-512 bytes), 1/32 per method description
        (64-256), 1/64 per step (40-160), budget / 1024 steps (3-6); at the
        service's 4,096-token budget 256 / 128 / 64 bytes and 4 steps."""
        b = max(0, int(budget))
        return cls(desc=int(desc) or min(512, max(96, b // 16)),
                   method=int(method) or min(256, max(64, b // 32)),
                   step=int(step) or min(160, max(40, b // 64)),
                   max_steps=int(max_steps) or min(6, max(3, b // 1024)))

    def scaled(self, scale: float) -> Tuple[Tuple[int, int], Tuple[int, int], Tuple[int, int]]:
        """(min, max) length pairs of the three strings at ``scale``."""
        def L(lo, hi):
            hi = max(4, int(hi * scale))
            return (min(lo, max(2, hi)), hi)
        return L(8, self.desc), L(6, self.method), L(4, self.step)


ReplyShape.LEGACY = ReplyShape(96, 64, 40, 3)


def _type_choice_segs(type_choice: bool) -> List[Segment]:
    """The classTypeCorrection value: the model's choice (null or one of the
    10 types), or a forced ``null`` -- an engine over random-initialised
    weights must not overwrite the statically inferred class types."""
    if type_choice:
        return [Segment(choice=CHOICE_CLASS_TYPE, then=[[]] * len(CHOICES[CHOICE_CLASS_TYPE]))]
    return [Segment(b"null")]


def build_template(names: Sequence[str], desc_len=(8, 96), method_len=(6, 64), step_len=(4, 40),
                   max_steps: int = 3, head: bool = True, type_choice: bool = True) -> List[Segment]:
    """Segments of one reply covering ``names``.  ``head`` = False: a
    continuation part (the description / correction come from part 0)."""
    if head:
        segs = [Segment(b'{"description": "'), Segment(None, *desc_len), Segment(b', "classTypeCorrection": ')]
        segs += _type_choice_segs(type_choice) + [Segment(b', "methods": [')]
    else:
        segs = [Segment(b'{"description": "", "classTypeCorrection": null, "methods": [')]
    for i, name in enumerate(names):
        segs.append(Segment(b'{"methodName": ' + json.dumps(name).encode() + b', "description": "'))
        segs.append(Segment(None, *method_len))
        segs.append(Segment(b', "businessLogic": ["'))
        segs += _steps_chain(step_len, max_steps)
        segs.append(Segment(b"}" + (b", " if i + 1 < len(names) else b"")))
    segs.append(Segment(b"]}"))
    return _merge(segs)


def template_budget(segs: Sequence[Segment]) -> int:
    """Upper bound of the reply's tokens (a token spells >= 1 byte)."""
    n = 0
    for s in segs:
        if s.forced is not None:
            n += len(s.forced)
        elif s.choice >= 0:
            n += max(len(a) + template_budget(t or []) for a, t in zip(CHOICES[s.choice], s.then or
                                                                       [[]] * len(CHOICES[s.choice])))
        else:
            n += s.max_len + 1
    return n


def plan_reply(names: Sequence[str], budget: int, shape: Optional[ReplyShape] = None,
               type_choice: bool = True) -> Tuple[List[List[Segment]], int]:
    """The reply parts of a class within ``budget`` tokens each, and the
    number of methods that fit in none.  One part when the whole reply fits
    (string lengths and step counts shrink first, down to half); otherwise
    the methods are split over continuation parts -- generated side by side
    from the same prompt and merged -- so no method is silently dropped."""
    shape = shape or ReplyShape.LEGACY
    names = list(dict.fromkeys(names))
    for scale, steps in ((1.0, shape.max_steps), (0.75, min(2, shape.max_steps)), (0.5, min(2, shape.max_steps))):
        segs = build_template(names, *shape.scaled(scale), steps, type_choice=type_choice)
        if template_budget(segs) <= budget:
            return [segs], 0
    lens = ((6, 48), (4, 32), (3, 20), 2)
    minimal = ((2, 16), (2, 12), (2, 8), 1)
    parts: List[List[Segment]] = []
    dropped = 0
    cur: List[str] = []

    def build(ns, head, ls=lens):
        return build_template(ns, ls[0], ls[1], ls[2], ls[3], head=head, type_choice=type_choice)
    for name in names:
        if template_budget(build(cur + [name], not parts)) <= budget:
            cur.append(name)
            continue
        if cur:
            parts.append(build(cur, not parts))
            cur = []
        if template_budget(build([name], not parts)) <= budget:
            cur = [name]
        elif template_budget(build([name], not parts, minimal)) <= budget:
            parts.append(build([name], not parts, minimal))
        else:
            dropped += 1
    if cur or not parts:
        segs = build(cur, not parts)
        if template_budget(segs) > budget:
            segs = build(cur, not parts, minimal)
        parts.append(segs)
    return parts, dropped


def build_head(has_methods: bool, desc_len=(8, 96), type_choice: bool = True) -> List[Segment]:
    """The class-level part of a reply generated with method branches: the
    description and the class-type choice, up to the opening of the methods
    list (or the whole reply when there is no method)."""
    return _merge([Segment(b'{"description": "'), Segment(None, *desc_len), Segment(b', "classTypeCorrection": ')]
                  + _type_choice_segs(type_choice)
                  + [Segment(b', "methods": [' if has_methods else b', "methods": []}')])


def build_branch(name: str, method_len=(6, 64), step_len=(4, 40), max_steps: int = 3) -> List[Segment]:
    """One method's entry, decoded as its own sequence after the class head
    (its first, empty segment stands for the prompt a branch never
    prefills: it continues the head's KV)."""
    body = [Segment(b'{"methodName": ' + json.dumps(name).encode() + b', "description": "'), Segment(None, *method_len),
            Segment(b', "businessLogic": ["')] + _steps_chain(step_len, max_steps) + [Segment(b"}")]
    return [Segment(b"")] + _merge(body)


def plan_branches(names: Sequence[str], budget: int, shape: Optional[ReplyShape] = None,
                  type_choice: bool = True) -> Tuple[List[Segment], List[List[Segment]]]:
    """(head, one branch per method) with string lengths and step counts
    shrunk until head + all branches fit ``budget`` tokens (down to a floor:
    no method is ever dropped -- past the floor the budget is exceeded)."""
    shape = shape or ReplyShape.LEGACY
    names = list(dict.fromkeys(names))
    plan = None
    ms = shape.max_steps
    for scale, steps in ((1.0, ms), (0.75, min(2, ms)), (0.5, min(2, ms)), (0.35, 1), (0.25, 1)):
        dl, ml, sl = shape.scaled(scale)
        head = build_head(bool(names), dl, type_choice=type_choice)
        branches = [build_branch(n, ml, sl, steps) for n in names]
        plan = (head, branches)
        if template_budget(head) + sum(template_budget(b) for b in branches) <= budget:
            break
    return plan


def _grammar_module():
    """``dmcp.enrich._grammar`` -- or the build ``DMCP_GRAMMAR_SO`` names
    (the ASan/UBSan one of scripts/asan_tests.sh)."""
    import os
    path = os.environ.get("DMCP_GRAMMAR_SO")
    if not path:
        from . import _grammar
        return _grammar
    import importlib.util
    import sys
    mod = sys.modules.get("dmcp.enrich._grammar")
    if mod is not None and getattr(mod, "__file__", None) == path:
        return mod
    spec = importlib.util.spec_from_file_location("dmcp.enrich._grammar", path)
    if spec is None:
        raise ImportError(f"DMCP_GRAMMAR_SO={path}: not a loadable module")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    sys.modules["dmcp.enrich._grammar"] = mod
    return mod


def _trim_to_word(out: bytearray, start: int) -> None:
    """A free string that reached its byte cap ends at its last word
    boundary, not mid-word: ``out[start:]`` (the string so far) is cut at
    its last space when that keeps at least half of it (trailing spaces
    dropped).  Only the reply text is cut; the KV cache keeps what was
    generated.  The native engine does the same (engine.cpp trim_to_word)."""
    body = out[start:]
    cut = body.rfind(b" ")
    if cut < max(1, len(body) // 2):
        return
    while cut > 0 and body[cut - 1] == 0x20:
        cut -= 1
    del out[start + cut:]


def merge_branches(head: str, branches: Sequence[str]) -> str:
    """The reply of a class decoded with method branches."""
    return head + ", ".join(branches) + ("]}" if branches else "")


def fit_template(inp: EnrichmentInput, capacity: int) -> List[Segment]:
    """The first part of :func:`plan_reply` (single-part callers)."""
    return plan_reply(inp.method_names, capacity)[0][0]


def merge_parts(raws: Sequence[str]) -> str:
    """One reply from the parts of a split class: part 0's description and
    correction, every part's methods in order."""
    head = json.loads(raws[0])
    for r in raws[1:]:
        head["methods"] = list(head.get("methods") or []) + list(json.loads(r).get("methods") or [])
    return json.dumps(head)


@dataclass
class _Seq:
    inp: EnrichmentInput
    index: Any                         # the caller's key
    segs: List[Segment]
    part: int = 0                      # reply part of a split class (plan_reply)
    n_parts: int = 1
    slot: int = -1
    pos: int = 0                       # tokens already in the KV cache
    seg: int = 0
    free_len: int = 0                  # tokens of the current free string
    free_bytes: int = 0                # ... and its bytes
    free_start: int = 0                # offset in ``out`` where the current free string starts
    forced_off: int = 0
    choice_pref: bytes = b""           # bytes chosen so far in the current choice segment
    next_token: int = -1               # token to feed at the next decode step
    next_src: int = -1                 # ... or: row of the last launched step whose selection it is
    await_row: int = -1                # ... or: a choice token selected at this row of step ``await_step``
    await_step: int = -1
    out: bytearray = field(default_factory=bytearray)
    done: bool = False
    prompt_tokens: int = 0
    gen_tokens: int = 0
    prompt: Optional[List[int]] = None   # prompt tokens ([BOS] + text)
    prefix_split: int = 0                # leading prompt tokens encoding the text before 'Source of'
    shared: bool = False                 # its prompt starts with the resident shared prefix (set at admission)
    h: int = -1                          # its state in the native grammar engine (-1: Python state)
    branches: Optional[List[List[Segment]]] = None  # a class head: its method branches (forked when it finishes)
    fork: Optional["_Fork"] = None       # a method branch: the fork it belongs to
    forked: bool = False                 # head or branch of a forked class (replies merge as branches)

    _free_budget: int = -1

    @property
    def free_budget(self) -> int:
        """Sampled (non-forced) tokens the reply may take: ~its decode steps
        (of the reply as planned; computed once -- the admission order key)."""
        if self._free_budget < 0:
            self._free_budget = template_budget([s for s in self.segs if s.forced is None]) + max(
                (template_budget([s for s in b if s.forced is None]) for b in self.branches or ()), default=0)
        return self._free_budget


@dataclass
class _Fork:
    """A class head's method branches.  The head's slot (the anchor) keeps
    the head's KV [0, pos); branch 0 continues in it, every other branch
    decodes in a slot of its own that reads the keys below ``pos`` from the
    anchor in place (``LocalLM.fork_share``: no copy), writing only past
    ``pos`` -- so a finished branch's slot, anchor or not, is a valid start
    for the next pending branch.  The anchor is released only when no
    running branch reads it any more."""
    head: "_Seq"
    pos: int
    pending: Deque[Tuple[int, List[Segment]]]
    holders: set = field(default_factory=set)   # slots of running branches
    anchor: int = -1                             # the head's slot
    anchor_held: bool = True                     # a running branch decodes in the anchor


class _IterClock:
    """Host time of the engine loop's iterations by phase, keeping the
    ``keep`` slowest (``LocalEngine.slow_iters``): an iteration whose host
    work outlasts the step queued ahead of it leaves the GPU idle, and which
    phase it spent that time in (refill, admission, step build, waits,
    replies) names the cause."""

    def __init__(self, keep: int = 5) -> None:
        self.keep = keep
        self.slow: List[Tuple[float, Dict[str, float]]] = []
        self._t0 = self._t = 0.0
        self._ph: Dict[str, float] = {}

    def next(self) -> None:
        """Closes the running iteration (if any) and starts the next."""
        now = time.perf_counter()
        if self._t0:
            self.lap("rest", now)
            total = 1e3 * (now - self._t0)
            if len(self.slow) < self.keep or total > self.slow[-1][0]:
                self.slow.append((round(total, 3), {k: round(1e3 * v, 3) for k, v in self._ph.items()}))
                self.slow.sort(key=lambda x: -x[0])
                del self.slow[self.keep:]
        self._t0 = self._t = now
        self._ph = {}

    def lap(self, name: str, now: float = 0.0) -> None:
        now = now or time.perf_counter()
        self._ph[name] = self._ph.get(name, 0.0) + now - self._t
        self._t = now


from .feeds import IterFeed, QueueFeed  # noqa: E402,F401  (re-exported)


PREFIX_MARKER = b"Source of "  # build_enrichment_prompt: everything before it is per-project


class LocalEngine:
    """Continuous-batching, grammar-constrained greedy generator over one LocalLM.

    :meth:`stream` is the engine: it pulls classes from a feed only while it
    has free KV slots (plus a small look-ahead), prefills every admitted
    class of a step in one batched prefill, and yields each reply the moment
    its sequence finishes -- the caller applies it while the GPU runs the
    next step.  :meth:`generate` is the list-in, list-out wrapper.

    The reply grammar (:func:`build_template`) forces the JSON skeleton and
    every extracted method name; the model writes the strings and makes the
    reference's choices (``ClaudeApiClient.java:101-120``): the class-type
    correction (``null`` or one of the 10 types) and when each method's
    business-logic list ends (1..3 steps).  A choice is sampled under the
    vocabulary mask of its trie state (tokens that keep the bytes a prefix
    of some alternative); once one alternative is left, its rest is forced.
    ``max_new_tokens`` bounds every reply (the reference's ``max_tokens``);
    a class whose methods do not fit is split into parts generated side by
    side and merged (:func:`plan_reply`) -- ``stats["methods_dropped"]``
    counts methods that fit in no part (a single method name longer than
    the budget).

    ``jump_forward``: forced skeleton bytes are not fed one per step -- after
    a sequence's token is fed, every following token that is already decided
    (the rest of a forced segment, or the closing quote of a string at its
    length cap) is appended to the SAME step as extra rows of that sequence,
    up to ``max_rows`` rows per step.  The KV append + causal per-row
    attention of :meth:`LocalLM.decode` makes that an exact multi-token
    extend, so only sampled tokens cost a step each.

    ``pipeline``: step t+1 is launched before step t's ids reach the host.
    A free-text row's token is gathered on the device from the previous
    step's selection; its mask assumes the token does not close the string,
    and the gather kernel switches it to the next segment's mask when it
    does (``mask_alt``).  A choice token's successor depends on which token
    it is, so that sequence sits out one step while the host reads it.

    ``shared_prefix``: the part of every prompt before ``Source of`` (the
    instructions + README of one project) is prefilled once into the
    model's prefix slot; decode reads it through the shared-prefix kernel.
    Several projects stream through one engine at once (feed items
    ``(key, input, readme)``): a class whose prompt does not start with the
    resident prefix -- another project, or a truncated prompt -- is admitted
    with its whole prompt in its own slot (its decode rows flagged off the
    prefix), and the prefix moves to the next project once no running
    sequence reads it.

    ``tokenizer``: the vocabulary of ``model`` (:mod:`dmcp.enrich.tokenizer`);
    default the byte-level one of the built-in presets.
    """

    MASK_NO_QUOTE, MASK_QUOTE = 0, 1
    MIN_SHARED_PREFIX = 64  # tokens; shorter common prefixes are not worth a separate prefill
    ADMIT_TOKENS = 32768    # prompt tokens per batched prefill (one GEMM per projection over all of them)
    ADMIT_SEQS = 64

    def __init__(self, model: LocalLM, use_graphs: bool = True, max_prompt_tokens: Optional[int] = None,
                 jump_forward: bool = True, shared_prefix: bool = True, pipeline: bool = True,
                 admit_min: Optional[int] = None, longest_first: bool = True, tokenizer=None,
                 max_new_tokens: Optional[int] = None, native_grammar: Optional[bool] = None,
                 fork_methods: bool = True, fork_max_context: int = 0,
                 reply_shape: Optional[ReplyShape] = None, type_choice: Optional[bool] = None,
                 precapture: Optional[bool] = None) -> None:
        self.model = model
        self.tok = tokenizer if tokenizer is not None else ByteTokenizer(model.cfg.vocab_size)
        self._tb = self.tok.token_bytes
        self._quote = self.tok.quote
        if len(self._tb) < model.cfg.vocab_size:  # ids the tokenizer does not name append nothing
            self._tb = list(self._tb) + [b""] * (model.cfg.vocab_size - len(self._tb))
        # admit the pending classes with the longest reply budget first (LPT):
        # the run's tail is then short replies, not a few long ones decoding
        # alone in a nearly empty batch
        self.longest_first = longest_first
        # a running batch admits new classes only once this many slots are
        # free (or nothing else is pending): every admission stalls the whole
        # decode batch for a prefill, so fewer, larger prefills (one GEMM per
        # projection over all their tokens) cost less than one per freed slot
        self.admit_min = max(1, admit_min if admit_min is not None else model.cfg.max_batch // 16)
        # method branches: once a class's head (description, class type) is
        # written, each method is decoded as its own sequence from a copy of
        # the head's KV -- a class's critical path is its head + its longest
        # method instead of all its methods in a row (small projects are
        # latency-bound: rows per step far below capacity)
        self.fork_methods = fork_methods
        # ... unless the class's own context (prompt after the shared prefix)
        # is longer than this (0: no limit, the default).  In round 4 forking
        # the byte-level preset's ~2,400-token classes lost in a full batch
        # (74.9 -> 69.8 classes/s, profiles/enrich_fork_context_ab_r4.jsonl);
        # with 768 slots and the per-row attention's kv-head-major items (a
        # class's branch rows, adjacent in the step, re-read the head's keys on
        # one CU) it wins: 42.3 -> 52.6 classes/s at 1,024 classes
        # (profiles/enrich_fork_context_ab_r5.txt)
        self.fork_max_context = int(fork_max_context)
        self.cfg: LMConfig = model.cfg
        # reply budget: the caller's max_new_tokens, within what the KV slot
        # leaves next to a useful prompt
        kv_cap = self.cfg.max_seq - max(64, self.cfg.max_seq // 4)
        self.reply_budget = min(kv_cap, int(max_new_tokens)) if max_new_tokens else kv_cap
        # string caps / step count of the replies (derived from the budget
        # unless given); a string at its cap closes at its last word boundary
        if isinstance(reply_shape, dict):  # config overrides (0 = derived), e.g. from a worker frame
            reply_shape = ReplyShape.from_budget(self.reply_budget, **reply_shape)
        self.reply_shape = reply_shape or ReplyShape.from_budget(self.reply_budget)
        # classTypeCorrection is the model's choice only for a loaded
        # checkpoint: random-initialised weights would overwrite the class
        # types found by static analysis with arbitrary ones (forced null)
        self.type_choice = bool(getattr(model, "checkpoint", None)) if type_choice is None else bool(type_choice)
        dev = model.device
        self._choice_rows: Dict[Tuple[int, bytes], int] = {}
        masks = list(self.tok.json_masks(self.cfg.vocab_size)) + self._choice_masks()
        self.masks = torch.tensor(masks, dtype=torch.int32, device=dev)
        self.graphs = DecodeGraphs(model, self.masks, alt_token=self._quote) \
            if use_graphs and dev.type == "cuda" else None
        # every row-count bucket's decode graph captured now, at engine start:
        # captured on first use instead, the larger buckets' captures (~15 ms
        # each, the GPU idle meanwhile) landed inside the first big run --
        # 23 % of the Llama-shape decode window (profiles/engine_gaps_r5.txt).
        # LOCAL_LLM_PRECAPTURE=0 restores capture on first use.
        if precapture is None:
            precapture = os.environ.get("LOCAL_LLM_PRECAPTURE", "1") != "0"
        if self.graphs is not None and precapture:
            self.graphs.capture_all()
        self.max_prompt_tokens = max_prompt_tokens
        self.jump_forward = jump_forward
        self.shared_prefix = shared_prefix and model.shared_prefix
        self.max_rows = model.max_rows
        self.pipeline = pipeline
        # classes taken from the feed per loop iteration (0 = all the free slots + look-ahead at once)
        self.refill_chunk = int(os.environ.get("LOCAL_LLM_REFILL_CHUNK", "32"))
        # fork-table rows applied once per decode launch (False: at each call)
        self.fork_batch = os.environ.get("LOCAL_LLM_FORK_BATCH", "1") != "0"
        # refill + admission under the launched step (see _session); 0 = at the iteration's top
        self.host_under_step = os.environ.get("LOCAL_LLM_HOST_UNDER_STEP", "1") != "0"
        # batched prefills that may be in flight at once
        self.admit_depth = max(1, int(os.environ.get("LOCAL_LLM_ADMIT_DEPTH", "2")))
        # previous step's selections for host-less gathers (graphs keep their own)
        self._last_ids = self.graphs.last_ids if self.graphs is not None else \
            torch.zeros(self.max_rows, dtype=torch.int32, device=dev)
        # pinned double buffer for the ids of the last two launched steps
        self._host_ids = [torch.zeros(self.max_rows, dtype=torch.int32, pin_memory=dev.type == "cuda")
                          for _ in range(2)]
        self.stats = {"prompt_tokens": 0, "generated_tokens": 0, "decode_steps": 0, "decode_rows": 0,
                      "prefills": 0, "prefill_batches": 0, "decode_s": 0.0, "prefill_s": 0.0, "prefix_tokens": 0,
                      "prefix_switches": 0, "unshared_prefills": 0,
                      "prefix_s": 0.0, "host_s": 0.0, "wait_s": 0.0, "launch_s": 0.0, "prefill_gpu_s": 0.0,
                      "reply_parts": 0,
                      "split_classes": 0, "methods_dropped": 0, "type_corrections": 0, "choice_waits": 0,
                      "forks": 0, "fork_branches": 0, "fork_waits": 0, "fork_skipped": 0,
                      "graph_replays": 0, "graph_kernels": 0, "under_s": 0.0}
        self._pf_events: List[tuple] = []  # (start, end) device events of the batched prefills
        self.slow_iters: List[Tuple[float, Dict[str, float]]] = []  # the last session's slowest loop iterations
        self._lock = threading.Lock()
        self._frag_cache: Dict[bytes, List[int]] = {}      # forced text -> ids
        self._prefix_cache: Dict[str, List[int]] = {}      # per-project prompt text -> ids (one project at a time)
        self._cont_cache: Dict[str, List[int]] = {}        # per-class prompt text -> ids (one admission's batch)
        # the grammar state machine + step builder in native code
        # (native/grammar/engine.cpp); None = the Python implementation below
        # (the reference: both give the same replies, tests/test_local_engine.py)
        self._native = self._make_native() if native_grammar is not False else None
        if native_grammar and self._native is None:
            raise RuntimeError("native grammar engine requested but dmcp.enrich._grammar is not built")
        import numpy as np
        self._stage = np.zeros((7, self.max_rows), dtype=np.int32)  # the native builder's step rows
        self._host_np = [h.numpy() for h in self._host_ids]
        self._ids_events = [torch.cuda.Event(), torch.cuda.Event()] if dev.type == "cuda" else [None, None]
        # the model, tokenizer (128k vocabulary entries) and tables built above
        # live as long as the engine: out of the cyclic collector's scans, so a
        # full collection during a run walks only the run's own objects (a
        # full scan paused the decode loop for tens of ms, GPU idle)
        if dev.type == "cuda" and os.environ.get("LOCAL_LLM_GC_FREEZE", "1") != "0":
            gc.collect()
            gc.freeze()
        # full collections wait this many young-generation passes during a
        # session (0 = the interpreter's own threshold); GPU only
        self.gc_full_every = int(os.environ.get("LOCAL_LLM_GC_FULL_EVERY", "1000")) if dev.type == "cuda" else 0

    def _count_graphs(self) -> None:
        """The device witness in the stats: hipGraph replays and the kernel
        nodes they launched (cumulative, like every engine stat)."""
        if self.graphs is not None:
            self.stats["graph_replays"] = self.graphs.counts["graph_replays"]
            self.stats["graph_kernels"] = self.graphs.counts["graph_kernels"]

    # ---------------------------------------------------------------- api
    def generate(self, inputs: Sequence[EnrichmentInput], readme: Optional[str]) -> List[str]:
        """Returns the raw JSON reply for every input (same order)."""
        out: Dict[int, str] = {}
        for i, raw in self.stream(enumerate(inputs), readme):
            out[i] = raw
        return [out[i] for i in range(len(inputs))]

    def stream(self, items, readme: Optional[str]) -> Iterator[Tuple[Any, str]]:
        """Yields ``(key, raw reply)`` as classes finish.  ``items``: an
        iterable of ``(key, EnrichmentInput)`` -- or ``(key, input, readme)``
        to mix projects -- or a feed of them (``take`` / ``done``)."""
        feed = items if hasattr(items, "take") else IterFeed(items)
        with self._lock:
            yield from self._session(feed, readme)

    # ------------------------------------------------------------ grammar
    def _make_native(self):
        try:
            _grammar = _grammar_module()
        except ImportError:
            return None
        rest = {}
        for cid, alts in CHOICES.items():
            for k, alt in enumerate(alts):
                for p in range(1, len(alt)):
                    rest[(cid, k, p)] = self._fragment(alt[p:])
        return _grammar.Engine(list(self._tb), int(self._quote), [list(CHOICES[c]) for c in sorted(CHOICES)],
                               dict(self._choice_rows), rest, self.jump_forward, self.pipeline, self.max_rows)

    def _native_template(self, segs: List[Segment]) -> int:
        """Registers ``segs`` (and the branch lists its choices splice in)."""
        lists: List[Optional[list]] = []
        index: Dict[int, int] = {}

        def add(lst: List[Segment]) -> int:
            if not lst:
                return -1
            if id(lst) in index:
                return index[id(lst)]
            i = len(lists)
            index[id(lst)] = i
            lists.append(None)
            spec = []
            for seg in self._encode_forced(lst):
                if seg.forced is not None:
                    spec.append((0, seg.ids, 0, 0, -1, []))
                elif seg.choice >= 0:
                    spec.append((2, [], 0, 0, seg.choice, [add(t) for t in (seg.then or [])]))
                else:
                    spec.append((1, [], seg.min_len, seg.max_len, -1, []))
            lists[i] = spec
            return i
        add(segs)
        return self._native.add_template(lists)

    def _choice_masks(self) -> List[List[int]]:
        """Mask rows of every choice trie state (appended after the two
        free-text rows); fills ``_choice_rows[(choice, prefix)]``."""
        from .tokenizer import _pack_bits
        rows: List[List[int]] = []
        V = self.cfg.vocab_size
        for cid, alts in CHOICES.items():
            chars = set(b"".join(alts))
            longest = max(len(a) for a in alts)
            cand = [(i, b) for i, b in enumerate(self._tb[:V])
                    if b and len(b) <= longest and all(c in chars for c in b)]
            prefixes = sorted({a[:k] for a in alts for k in range(len(a))})
            for p in prefixes:
                ok = [i for i, b in cand if any(a.startswith(p + b) for a in alts)]
                if not ok:
                    raise ValueError(f"tokenizer cannot spell choice {alts!r} after {p!r}")
                self._choice_rows[(cid, p)] = 2 + len(rows)
                rows.append(_pack_bits(ok, V))
        return rows

    def _enter(self, s: _Seq) -> Optional[int]:
        """Moves ``s`` into its current segment: a forced token becomes
        ``next_token`` (returns None), a free string or a choice returns the
        mask row of its first selection; past the last segment ``s`` is done."""
        while s.seg < len(s.segs):
            seg = s.segs[s.seg]
            if seg.forced is not None:
                if s.forced_off < len(seg.ids):
                    s.next_token = seg.ids[s.forced_off]
                    s.forced_off += 1
                    return None
                s.seg += 1
                s.forced_off = 0
                continue
            if seg.choice >= 0:
                s.choice_pref = b""
                return self._choice_rows[(seg.choice, b"")]
            s.free_len = s.free_bytes = 0
            s.free_start = len(s.out)
            return self.MASK_QUOTE if seg.min_len == 0 else self.MASK_NO_QUOTE
        s.done = True
        return None

    def _choose(self, s: _Seq, seg: Segment, k: int, rest: bytes) -> Optional[int]:
        """Alternative ``k`` of the choice at ``s.seg`` is decided: its
        remaining bytes ``rest`` are forced, its branch spliced in."""
        after: List[Segment] = []
        if rest:
            after.append(Segment(rest, ids=self._fragment(rest)))
        if seg.then and seg.then[k]:
            after += self._encode_forced(list(seg.then[k]))
        if seg.choice == CHOICE_CLASS_TYPE and k > 0:
            self.stats["type_corrections"] += 1
        s.segs = s.segs[:s.seg + 1] + after + s.segs[s.seg + 1:]
        s.seg += 1
        s.forced_off = 0
        return self._enter(s)

    def _after_feed(self, s: _Seq, tok: int) -> Optional[int]:
        """Grammar transition after ``tok`` entered the KV cache.  Returns
        None when the next token is already decided (``s.next_token``) or the
        reply is complete, else the mask row of the selection at this row."""
        s.out += self._tb[tok]
        s.pos += 1
        s.gen_tokens += 1
        seg = s.segs[s.seg] if s.seg < len(s.segs) else None
        if seg is None:
            return self._enter(s)
        if seg.forced is not None:
            return self._enter(s)
        if seg.choice >= 0:
            pref = s.choice_pref + self._tb[tok]
            alts = CHOICES[seg.choice]
            live = [k for k, a in enumerate(alts) if a.startswith(pref)]
            if not live:  # cannot happen under the choice masks
                raise RuntimeError(f"token {tok} leaves choice {alts!r} after {s.choice_pref!r}")
            if len(live) == 1:
                k = live[0]
                return self._choose(s, seg, k, alts[k][len(pref):])
            s.choice_pref = pref
            return self._choice_rows[(seg.choice, pref)]
        if tok == self._quote:  # free string closed
            s.seg += 1
            s.forced_off = 0
            s.free_len = 0
            return self._enter(s)
        s.free_len += 1
        s.free_bytes += len(self._tb[tok])
        if s.free_bytes >= seg.max_len:
            _trim_to_word(s.out, s.free_start)
            s.next_token = self._quote
            return None
        return self.MASK_QUOTE if s.free_len >= seg.min_len else self.MASK_NO_QUOTE

    def _in_choice(self, s: _Seq) -> bool:
        return not s.done and s.seg < len(s.segs) and s.segs[s.seg].choice >= 0

    def _speculative_mask(self, s: _Seq) -> Tuple[int, int]:
        """(mask row, mask row if the token is the closing quote) of a row
        whose free-text token is still on the device: the state after
        feeding any token but the quote, and the first mask of the segment
        the quote opens when that is a choice (-1: its selection is unused)."""
        seg = s.segs[s.seg]
        main = self.MASK_QUOTE if s.free_len + 1 >= seg.min_len else self.MASK_NO_QUOTE
        alt = -1
        if s.seg + 1 < len(s.segs):
            nxt = s.segs[s.seg + 1]
            if nxt.choice >= 0:
                alt = self._choice_rows[(nxt.choice, b"")]
            elif nxt.forced is None:
                alt = self.MASK_QUOTE if nxt.min_len == 0 else self.MASK_NO_QUOTE
        return main, alt

    # ------------------------------------------------------------ helpers
    def _prompt(self, seq: _Seq, readme: Optional[str], budget: int) -> List[int]:
        """Prompt tokens of ``seq``; sets ``seq.prefix_split``."""
        text = build_enrichment_prompt(seq.inp, readme)
        i = text.find(PREFIX_MARKER.decode())
        if i > 0:  # the per-project text (instructions + README) is tokenised once per project
            pre = self._prefix_cache.get(text[:i])
            if pre is None:
                if len(self._prefix_cache) >= 8:
                    self._prefix_cache.clear()
                pre = self._prefix_cache[text[:i]] = ([self.tok.bos] if self.tok.bos is not None else []) + \
                    self.tok.encode(text[:i])
            cont = self._cont_cache.get(text[i:])  # pre-tokenised with its admission's batch
            ids, split = pre + (cont if cont is not None else self.tok.encode_continuation(text[i:])), len(pre)
        else:
            ids, split = self.tok.encode_split(text, PREFIX_MARKER.decode())
        head = 1 if self.tok.bos is not None else 0
        limit = self.cfg.max_seq - budget - 2
        if self.max_prompt_tokens:
            limit = min(limit, self.max_prompt_tokens)
        if limit < 16:
            raise ValueError("KV capacity too small for the reply template")
        if len(ids) - head > limit:
            keep_tail = min(256, limit // 4)  # keep the instructions at the end
            cut = head + limit - keep_tail
            ids = ids[:cut] + ids[len(ids) - keep_tail:]
            if split > cut:  # the marker was cut out: no shared prefix
                split = 0
        seq.prefix_split = split
        return ids

    def _pretokenize(self, items, readme: Optional[str]) -> None:
        """The per-class parts of the prompts of ``items`` (feed items: key,
        input[, readme]) in one batched tokenizer call, for :meth:`_prompt`.
        One class at a time, a 128k-id BPE tokenised ~1.2 ms per prompt on
        the engine thread -- 60-80 ms per admission with the GPU idle
        (profiles/engine_gaps_r5.txt); the batch runs on the tokenizer's
        thread pool."""
        if len(items) < 2 or type(self.tok).encode_continuation_batch is _TokBase.encode_continuation_batch:
            return
        marker = PREFIX_MARKER.decode()
        todo = []
        for item in items:
            text = build_enrichment_prompt(item[1], item[2] if len(item) > 2 else readme)
            i = text.find(marker)
            if i > 0 and text[i:] not in self._cont_cache:
                todo.append(text[i:])
        if len(todo) > 1:
            self._cont_cache.update(zip(todo, self.tok.encode_continuation_batch(todo)))

    def _seq_prefix_len(self, s: _Seq) -> int:
        """Tokens of ``s.prompt`` before its per-class part, or 0."""
        P = s.prefix_split if self.shared_prefix else 0
        return P if self.MIN_SHARED_PREFIX <= P < len(s.prompt) else 0

    def _fragment(self, text: bytes) -> List[int]:
        ids = self._frag_cache.get(text)
        if ids is None:
            ids = self._frag_cache[text] = self.tok.encode_fragment(text.decode("utf-8"))
        return ids

    def _encode_forced(self, segs: List[Segment]) -> List[Segment]:
        for seg in segs:
            if seg.forced is not None and seg.ids is None:
                seg.ids = self._fragment(seg.forced)
        return segs

    def _build_prompt(self, s: _Seq, readme: Optional[str]) -> List[int]:
        budget = template_budget(s.segs)
        if budget + 32 > self.cfg.max_seq:
            raise ValueError(f"reply template needs {budget} tokens > max_seq {self.cfg.max_seq}")
        return self._prompt(s, readme, budget)

    def _seqs_for(self, key: Any, inp: EnrichmentInput, readme: Optional[str], small: bool = False) -> List[_Seq]:
        """The sequences of one class: one per reply part, sharing one prompt --
        or, with ``fork_methods``, its head (the branches follow its KV).
        ``small``: the session's batch is latency-bound, fork whatever the
        class's own context length."""
        if self.fork_methods:
            head, branches = plan_branches(inp.method_names, self.reply_budget, self.reply_shape, self.type_choice)
            q = _Seq(inp, key, self._encode_forced(head), part=0, n_parts=1 + len(branches))
            q.branches = [self._encode_forced(b) for b in branches] if branches else None
            self.stats["reply_parts"] += 1
            if self._native is not None:
                q.h = self._native.new_seq(self._native_template(q.segs))
            try:
                longest = max((template_budget(b) for b in branches), default=0)
                q.prompt = self._prompt(q, readme, template_budget(head) + longest)
            except BaseException:
                if q.h >= 0:
                    self._native.release(q.h)
                raise
            if not branches or not self.fork_max_context or small or \
                    len(q.prompt) - q.prefix_split <= self.fork_max_context:
                q.forked = True
                return [q]
            if q.h >= 0:  # a long own context: its methods decode in one sequence
                self._native.release(q.h)
            self.stats["reply_parts"] -= 1
            self.stats["fork_skipped"] += 1
        parts, dropped = plan_reply(inp.method_names, self.reply_budget, self.reply_shape, self.type_choice)
        self.stats["methods_dropped"] += dropped
        self.stats["reply_parts"] += len(parts)
        if len(parts) > 1:
            self.stats["split_classes"] += 1
        if dropped:
            LOG.warning("%s: %d method(s) do not fit a %d-token reply", inp.full_class_name, dropped,
                        self.reply_budget)
        seqs = [_Seq(inp, key, self._encode_forced(segs), part=j, n_parts=len(parts))
                for j, segs in enumerate(parts)]
        if self._native is not None:
            try:
                for q in seqs:
                    q.h = self._native.new_seq(self._native_template(q.segs))
            except BaseException:
                for q in seqs:
                    if q.h >= 0:
                        self._native.release(q.h)
                raise
        # every part has the same prompt: tokenise once, sized for the longest reply
        longest = max(seqs, key=lambda q: template_budget(q.segs))
        prompt = self._build_prompt(longest, readme)
        for q in seqs:
            q.prompt, q.prefix_split = prompt, longest.prefix_split
        return seqs

    def _admit_batch(self, batch: List[_Seq]) -> List[_Seq]:
        """Prefills ``batch`` and waits for it (see :meth:`_admit_launch`);
        returns the sequences that finished already."""
        return self._admit_finish(self._admit_launch(batch), wait=True)

    def _admit_launch(self, batch: List[_Seq]) -> dict:
        """Enqueues ONE batched prefill of every sequence of ``batch`` (slots
        assigned) -- prompt + first forced segment, after the shared prefix
        for the sequences that use it -- and the masked argmax of each first selection; the ids
        land in a pinned buffer.  Nothing here waits for the device: the host
        goes on to build and launch the running batch's next step, which the
        stream runs after the prefill; the admitted classes join the step
        after that.  (The prefill on a second stream, overlapped with the
        decode steps, measured no faster: the two do not run concurrently to
        any useful degree -- profiles/overlap_prefill_r3.txt.)"""
        from .. import ops
        t0 = time.perf_counter()
        reqs = []
        need, midx_l = [], []
        for i, s in enumerate(batch):
            first = s.segs[0].ids or []
            toks = s.prompt + first
            start = self.model.fork_prefix(s.slot) if s.shared else 0
            if not s.shared:
                self.stats["unshared_prefills"] += 1
            reqs.append((toks[start:], s.slot, start))
            self.stats["prompt_tokens"] += len(toks) - start
            s.prompt_tokens = len(s.prompt)
            s.pos = len(toks)
            if s.h >= 0:
                m = self._native.admit(s.h, s.slot, s.pos, s.shared)
                m = None if m < 0 else m
            else:
                s.out.extend(s.segs[0].forced or b"")
                s.seg, s.forced_off = 1, 0
                m = self._enter(s)  # the first selection's mask, or a decided token
            if m is not None:
                need.append(i)
                midx_l.append(m)
        dev = self.model.device
        h = {"batch": batch, "need": need, "ids": None, "event": None}
        timed = dev.type == "cuda"
        if timed:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        logits = self.model.prefill_batch(reqs)  # [n, vocab]
        if timed:
            ev[1].record()
            self._pf_events.append(ev)
        if need:
            rows = logits[need] if len(need) < len(batch) else logits
            midx = torch.tensor(midx_l, dtype=torch.int32)
            if dev.type == "cuda":  # no pageable (host-blocking) copy behind the prefill
                midx = midx.pin_memory()
            midx = midx.to(dev, non_blocking=True)
            ids = ops.masked_argmax(rows.contiguous(), self.masks, vocab=self.cfg.vocab_size, mask_idx=midx)
            host = torch.empty(len(need), dtype=torch.int32, pin_memory=dev.type == "cuda")
            host.copy_(ids, non_blocking=dev.type == "cuda")
            h["ids"] = host
        if dev.type == "cuda":
            h["event"] = torch.cuda.Event()
            h["event"].record()
        self.stats["prefill_s"] += time.perf_counter() - t0
        return h

    def _admit_finish(self, h: dict, wait: bool) -> Optional[List[_Seq]]:
        """None while the prefill of ``h`` is still running (``wait=False``);
        else applies the first selections and returns the sequences that
        finished already (all forced)."""
        ev = h["event"]
        if ev is not None:
            if not wait and not ev.query():
                return None
            t0 = time.perf_counter()
            ev.synchronize()
            self.stats["prefill_s"] += time.perf_counter() - t0
        batch = h["batch"]
        nat = self._native
        if h["ids"] is not None:
            for i, tok in zip(h["need"], h["ids"].tolist()):
                if nat is not None:
                    nat.set_next(batch[i].h, int(tok))
                else:
                    batch[i].next_token = int(tok)
        if nat is not None:
            for s in batch:
                s.done = nat.is_done(s.h)
                if not s.done:
                    nat.activate(s.h)
        done = [s for s in batch if s.done]
        self.stats["prefills"] += len(batch)
        self.stats["prefill_batches"] += 1
        self._drain_prefill_events()
        return done

    def _drain_prefill_events(self) -> None:
        """Device time of the batched prefills that have finished, into
        ``prefill_gpu_s`` as they finish (a worker's per-project stats are
        deltas taken while its engine stream keeps running)."""
        while self._pf_events and self._pf_events[0][1].query():
            a, b = self._pf_events.pop(0)
            self.stats["prefill_gpu_s"] += a.elapsed_time(b) * 1e-3

    def _launch_staged(self, n: int, buf: int):
        """:meth:`_launch` of the native builder's rows (``self._stage[:, :n]``)."""
        self.model.fork_flush()  # this iteration's fork-table rows, one copy ahead of the step
        if self.graphs is not None:
            self.graphs.run_staged(self._stage, n)
            ids = self.graphs.last_ids
        else:
            t = torch.from_numpy(self._stage[:, :n].copy()).to(self.model.device)
            _, ids = self.model.decode_select_gather(t[0].contiguous(), t[4].contiguous(), self._last_ids,
                                                     t[1].contiguous(), t[2].contiguous(), self.masks,
                                                     t[3].contiguous(), t[5].contiguous(), self._quote,
                                                     t[6].contiguous())
        host = self._host_ids[buf]
        host[:n].copy_(ids[:n], non_blocking=self.model.device.type == "cuda")
        if self.model.device.type == "cuda":
            ev = self._ids_events[buf]  # reused: the step that last recorded it was waited for
            ev.record()
            return ev
        return None

    def _launch(self, toks: List[int], slots: List[int], poss: List[int], mrows: List[int],
                srcs: List[int], alts: List[int], prows: List[int], buf: int):
        """Launches one step; enqueues the copy of its ids to pinned buffer
        ``buf``; returns the event that completes with that copy."""
        self.model.fork_flush()
        if self.graphs is not None:
            _, ids = self.graphs.run(toks, slots, poss, mrows, srcs, alts, prows)
        else:
            dev = self.model.device
            t = torch.tensor([toks, slots, poss, mrows, srcs, alts, prows], dtype=torch.int32, device=dev)
            _, ids = self.model.decode_select_gather(t[0].contiguous(), t[4].contiguous(), self._last_ids,
                                                     t[1].contiguous(), t[2].contiguous(), self.masks,
                                                     t[3].contiguous(), t[5].contiguous(), self._quote,
                                                     t[6].contiguous())
        n = len(toks)
        host = self._host_ids[buf]
        host[:n].copy_(ids[:n], non_blocking=self.model.device.type == "cuda")
        if self.model.device.type == "cuda":
            ev = self._ids_events[buf]  # reused: the step that last recorded it was waited for
            ev.record()
            return ev
        return None

    def _finish(self, s: _Seq, partials: Dict[Any, List[Optional[str]]]) -> Optional[str]:
        """The class reply once ``s`` (a part of it) is complete, else None."""
        if s.h >= 0:
            raw = self._native.out(s.h).decode("utf-8", "replace")
            self._native.release(s.h)
            s.h = -1
        else:
            raw = s.out.decode("utf-8", "replace")
        if s.n_parts == 1:
            return raw
        got = partials.setdefault(s.index, [None] * s.n_parts)
        got[s.part] = raw
        if any(r is None for r in got):
            return None
        del partials[s.index]
        if s.forked:
            return merge_branches(got[0], got[1:])  # type: ignore[arg-type]
        return merge_parts(got)  # type: ignore[arg-type]

    def _start_branches(self, st: "_Fork", slots: List[int], src: Optional[int]) -> List[_Seq]:
        """Starts the next pending branches of ``st`` in ``slots`` -- with a copy
        of the head's own KV from sibling slot ``src`` (None: the slots
        already hold it: the head's, or a finished sibling's) -- admitted."""
        head, pos = st.head, st.pos
        kids = []
        for slot in slots:
            j, segs = st.pending.popleft()
            q = _Seq(head.inp, head.index, segs, part=1 + j, n_parts=head.n_parts)
            q.slot, q.pos, q.fork, q.forked = slot, pos, st, True
            q.shared, q.prompt, q.prefix_split = head.shared, head.prompt, head.prefix_split
            kids.append(q)
        share = [q.slot for q in kids if q.slot != st.anchor]
        if share:  # the branches' keys below pos: the anchor's, read in place
            self.model.fork_share(st.anchor, share, pos)
        nat = self._native
        for q in kids:
            if nat is not None:
                q.h = nat.new_seq(self._native_template(q.segs))
                m = nat.admit(q.h, q.slot, q.pos, q.shared)
                q.done = nat.is_done(q.h)
                if not q.done:
                    nat.activate(q.h)
            else:
                q.seg, q.forced_off = 1, 0
                m = self._enter(q)
            if m is not None and m >= 0:
                raise RuntimeError("a method branch must start with forced text")
            st.holders.add(q.slot)
        self.stats["fork_branches"] += len(kids)
        return kids

    # ------------------------------------------------------------ the loop
    def _session(self, feed, readme: Optional[str]):
        """Runs ``feed`` to its end (``readme``: the default of items without one).

        Each iteration: refill the look-ahead from the feed, admit (batched
        prefill) while KV slots are free, build step k's rows, launch it, then
        -- while the GPU computes step k -- wait for step k-1's ids, run the
        grammar transitions they decide and yield the finished replies.
        With ``pipeline`` a sequence whose next token is step k-1's free-text
        selection gets ONE row gathered on the device from that selection;
        a sequence whose next token is a choice selection sits out until the
        host has read it; every other sequence gets its literal token and,
        with jump-forward, the decided tokens after it.  Without ``pipeline``
        the host waits for every step's ids before building the next (the
        exact reference loop)."""
        cfg = self.cfg
        free_slots = list(range(cfg.max_batch - 1, -1, -1))
        pending: Deque[_Seq] = deque()
        active: List[_Seq] = []
        partials: Dict[Any, List[Optional[str]]] = {}
        lookahead = max(4, cfg.max_batch // 4)
        prefix_toks: Optional[List[int]] = None  # the resident shared prefix
        P = 0
        prev_event = None
        prev_buf, prev_n = 1, 0
        step_no = -1                     # number of the last launched step
        finished: List[_Seq] = []
        admits: Deque[dict] = deque()  # the batched prefills in flight, oldest first
        forks: List[_Fork] = []  # forks with branches still waiting for a slot
        nat0 = self._native
        self.model.fork_reset()  # no slot reads another's keys (a session left by an error included)
        # branch starts and slot releases only collect their fork-table rows;
        # each decode launch applies them in one copy (they came one small
        # copy + write per call, ~40 us of host each, thousands per run)
        self.model.fork_defer = self.fork_batch

        def release(slots: List[int]) -> None:
            """Slots back to the free list, owning all their keys again."""
            if slots:
                self.model.fork_clear(slots)
                free_slots.extend(slots)

        def fill(st: _Fork) -> None:
            """Pending branches of ``st`` into free slots (reading the anchor in place)."""
            k = min(len(st.pending), len(free_slots))
            if k and st.holders:
                active.extend(q for q in self._start_branches(st, [free_slots.pop() for _ in range(k)], st.anchor)
                              if not q.done)

        def retire(q: _Seq) -> None:
            """A finished sequence: its slot back -- or to a branch of its
            class -- and its text to the result."""
            st = q.fork
            if q.branches:  # a head: branch 0 continues in its slot, the anchor
                st = _Fork(q, nat0.pos(q.h) if nat0 is not None else q.pos, deque(enumerate(q.branches)),
                           anchor=q.slot)
                self.stats["forks"] += 1
                active.extend(k for k in self._start_branches(st, [q.slot], None) if not k.done)
                fill(st)
                if st.pending:
                    forks.append(st)
                elif not st.holders:  # every branch finished at once
                    release([q.slot])
            elif st is not None:  # a branch: a pending sibling takes its slot as it is
                st.holders.discard(q.slot)
                if st.pending:
                    active.extend(k for k in self._start_branches(st, [q.slot], None) if not k.done)
                else:
                    out = []
                    if q.slot == st.anchor:
                        st.anchor_held = False  # kept while other branches read it
                    else:
                        out.append(q.slot)
                    if not st.holders and not st.anchor_held:
                        out.append(st.anchor)  # the last reader finished
                    release(out)
            else:
                release([q.slot])
            finished.append(q)
        # the run's own objects (segments, sequences, the caller's inputs:
        # ~10^5) are not frozen, and a full collection over them paused the
        # loop for 25-45 ms, GPU idle, about once per run
        # (profiles/engine_gc_r5.txt): the session defers full collections
        # (young ones still run; refcounting frees everything acyclic)
        gc_deferred = bool(self.gc_full_every)
        if gc_deferred:
            _gc_defer_enter(self.gc_full_every)
        clock = _IterClock()

        def refill():
            """Tops up the look-ahead from the feed (blocking only when idle);
            returns whether the feed had a whole chunk ready (more may wait).
            Yields the error replies of classes that cannot be set up."""
            nonlocal pending
            want = len(free_slots) + lookahead - len(pending)
            if want <= 0 or feed.done:
                return False
            if self.refill_chunk > 0:
                # a chunk per iteration: its prompts' tokenisation and
                # sequence set-up (~0.2 ms a class) stay under the GPU work
                # already queued -- a step, or at the start the first
                # admissions' prefills -- instead of one refill of the whole
                # batch with the GPU idle (~180 ms per start at 768 slots,
                # profiles/engine_host_r5.txt)
                want = min(want, self.refill_chunk)
            items = list(feed.take(want, wait=not active and not pending and not admits))
            # a small batch -- the feed drained and every class fits in 3/4 of
            # the slots -- is latency-bound: long-context classes fork too
            # (profiles/enrich_fork_context_ab_r4.jsonl)
            small = len(items) < want and len(active) + len(pending) + len(items) <= cfg.max_batch * 3 // 4
            try:
                self._pretokenize(items, readme)
            except Exception:  # noqa: BLE001 -- each class then tokenises (and reports) on its own
                LOG.debug("batched prompt tokenisation failed", exc_info=True)
            for item in items:
                key, inp = item[0], item[1]
                try:
                    seqs = self._seqs_for(key, inp, item[2] if len(item) > 2 else readme, small)
                except Exception as e:
                    yield key, json.dumps({"error": str(e)})
                    continue
                pending.extend(seqs)
            self._cont_cache.clear()
            clock.lap("refill")
            return len(items) == want

        def admit() -> None:
            """One batched prefill for all that fit (up to admit_depth in flight:
            the next one's host work -- prompts, packing, ~130 launches -- runs
            under the previous one's prefill instead of after it, GPU idle)."""
            nonlocal pending, prefix_toks, P
            if not (len(admits) < self.admit_depth and pending and free_slots and (
                    not active or len(free_slots) >= self.admit_min
                    or (feed.done and len(free_slots) >= len(pending)))):
                return
            batch: List[_Seq] = []
            ntok = 0
            if self.longest_first and len(pending) > 1:
                pending = deque(sorted(pending, key=lambda q: -q.free_budget))
            # the resident prefix's readers: running and still prefilling
            users = sum(1 for q in active if q.shared) + \
                sum(1 for h in admits for q in h["batch"] if q.shared)
            while pending and free_slots and len(batch) < self.ADMIT_SEQS:
                s = pending[0]
                if self.shared_prefix and users == 0:
                    # no running sequence reads the resident prefix: it moves
                    # to this class's project
                    Ps = self._seq_prefix_len(s)
                    if Ps and s.prompt[:Ps] != prefix_toks:
                        t0 = time.perf_counter()
                        self.model.set_prefix(s.prompt[:Ps])
                        prefix_toks, P = s.prompt[:Ps], Ps
                        self.stats["prefix_s"] += time.perf_counter() - t0
                        self.stats["prefix_tokens"] += Ps
                        self.stats["prefix_switches"] += 1
                s.shared = bool(P) and len(s.prompt) > P and s.prompt[:P] == prefix_toks
                nxt = len(s.prompt) - (P if s.shared else 0)
                if batch and ntok + nxt > self.ADMIT_TOKENS:
                    break
                pending.popleft()
                s.slot = free_slots.pop()
                batch.append(s)
                users += s.shared
                ntok += nxt
            admits.append(self._admit_launch(batch))
            clock.lap("admit_launch")

        more = False  # the last refill found a whole chunk ready: more may be waiting
        try:
            while True:
                clock.next()
                # with a running batch the look-ahead refill and the next
                # admission run right after the step is launched, under it and
                # the one before (at the top of the iteration they ran with at
                # most one step queued: the GPU idled ~10 ms behind each
                # admission's ~17 ms of host work, profiles/engine_gaps_r6_*.txt)
                under = self.host_under_step and bool(active) and self.pipeline
                if not under:
                    more = yield from refill()
                if not pending and not active and not admits:
                    if feed.done:
                        break
                    continue
                # ---- branches of finished heads first (their classes are
                # further along than any class still to be admitted)
                for st in forks:
                    fill(st)
                forks = [st for st in forks if st.pending]
                clock.lap("forks")
                if not under:
                    admit()
                if admits:
                    # nothing decodes yet: keep preparing the feed while the
                    # first prefills run rather than wait for them
                    can_admit = len(admits) < self.admit_depth and pending and free_slots
                    done = self._admit_finish(admits[0], wait=not active and not more and not can_admit)
                    clock.lap("admit_finish")
                    if done is not None:
                        active.extend(s for s in admits.popleft()["batch"] if not s.done)
                        for s in done:
                            retire(s)
                        while finished:
                            s = finished.pop()
                            raw = self._finish(s, partials)
                            if raw is not None:
                                yield s.index, raw
                        continue  # admit the next batch before this step when slots allow
                if not active:
                    continue
                nat = self._native
                if nat is not None:  # ---- one step on the native grammar engine
                    t0 = time.perf_counter()
                    n = nat.build(self._stage, step_no + 1)
                    t1 = time.perf_counter()
                    event, buf = None, None
                    if n:
                        buf = 1 - prev_buf
                        event = self._launch_staged(n, buf)
                        step_no += 1
                    t2 = time.perf_counter()
                    if under:  # the refill / admission host work, under the steps in flight
                        clock.lap("build", t1)
                        clock.lap("launch", t2)
                        more = yield from refill()
                        admit()
                    th = time.perf_counter()
                    if not self.pipeline:
                        if event is not None:
                            event.synchronize()
                        nat.apply(self._host_np[buf][:n], step_no, step_no)
                    else:
                        # the ids of the step before the one just launched (or
                        # of the last one, when none was): the gathered rows'
                        # tokens and the awaited choices
                        if prev_event is not None:
                            prev_event.synchronize()
                        nat.apply(self._host_np[prev_buf][:prev_n], step_no - 1 if n else step_no, step_no)
                    t3 = time.perf_counter()
                    if n:
                        prev_event, prev_buf, prev_n = event, buf, n
                        self.stats["decode_steps"] += 1
                        self._count_graphs()
                        self.stats["decode_rows"] += n
                        self.stats["generated_tokens"] += n
                    fin = nat.collect_done()
                    if fin:
                        byh = {q.h: q for q in active}
                        for hh in fin:
                            byh[hh].done = True
                        active = [q for q in active if not q.done]
                        for hh in fin:
                            retire(byh[hh])
                    t4 = time.perf_counter()
                    if not under:
                        clock.lap("build", t1)
                        clock.lap("launch", t2)
                    clock.lap("wait", t3)
                    clock.lap("retire", t4)
                    self.stats["wait_s"] += t3 - th
                    self.stats["launch_s"] += t2 - t1
                    self.stats["host_s"] += (t1 - t0) + (t4 - t3) + (t2 - t1)
                    self.stats["decode_s"] += (t4 - t0) - (th - t2)  # the refill / admission are not the step's
                    self.stats["under_s"] += th - t2
                    for k, v in nat.stats().items():  # (cheap) so a never-ending worker stream reports them
                        self.stats[k] += v
                    nat.reset_stats()
                    while finished:
                        s = finished.pop()
                        raw = self._finish(s, partials)
                        if raw is not None:
                            yield s.index, raw
                    continue
                # ---- build and launch one step
                t0 = time.perf_counter()
                toks: List[int] = []
                slots: List[int] = []
                poss: List[int] = []
                mrows: List[int] = []
                srcs: List[int] = []
                alts: List[int] = []
                prows: List[int] = []
                gathered: List[Tuple[_Seq, int, int]] = []  # (seq, row, source row of the previous step)
                sample_at: List[Tuple[_Seq, int]] = []
                spare = self.max_rows - len(active)
                for s in active:
                    if s.await_row >= 0:
                        continue  # its next token is a choice selection the host has not read yet
                    if s.next_src >= 0:
                        gathered.append((s, len(toks), s.next_src))
                        m, a = self._speculative_mask(s)
                        toks.append(0)
                        slots.append(s.slot)
                        poss.append(s.pos)
                        mrows.append(m)
                        srcs.append(s.next_src)
                        alts.append(a)
                        prows.append(1 if s.shared else 0)
                        s.next_src = -1
                        continue
                    tok = s.next_token
                    while True:
                        toks.append(tok)
                        slots.append(s.slot)
                        poss.append(s.pos)
                        mrows.append(self.MASK_NO_QUOTE)
                        srcs.append(-1)
                        alts.append(-1)
                        prows.append(1 if s.shared else 0)
                        m = self._after_feed(s, tok)
                        if s.done:
                            break
                        if m is not None:  # this row's selection is the next token
                            mrows[-1] = m
                            if not self.pipeline:
                                sample_at.append((s, len(toks) - 1))
                            elif self._in_choice(s):
                                s.await_row, s.await_step = len(toks) - 1, step_no + 1
                            else:
                                s.next_src = len(toks) - 1
                            break
                        if not self.jump_forward or spare <= 0:
                            break
                        spare -= 1
                        tok = s.next_token
                t1 = time.perf_counter()
                if toks:
                    buf = 1 - prev_buf
                    event = self._launch(toks, slots, poss, mrows, srcs, alts, prows, buf)
                    step_no += 1
                else:  # every active sequence waits for a choice of the last step
                    event, buf = None, None
                t2 = time.perf_counter()
                if under:  # the refill / admission host work, under the steps in flight
                    more = yield from refill()
                    admit()
                th = time.perf_counter()
                if not self.pipeline:
                    if event is not None:
                        event.synchronize()
                    ids = self._host_ids[buf][:len(toks)].tolist()  # one conversion, not one per row
                    for s, r in sample_at:
                        s.next_token = ids[r]
                else:
                    # the ids of the step before the one just launched (or of
                    # the last one, when none was): gathered rows' tokens and
                    # awaited choices
                    read_no = step_no - 1 if toks else step_no
                    waiting = [s for s in active if s.await_row >= 0 and s.await_step == read_no]
                    if gathered or waiting:
                        if prev_event is not None:  # the step whose ids are read
                            prev_event.synchronize()
                        ids = self._host_ids[prev_buf][:prev_n].tolist()  # one conversion, not one per row
                        for s in waiting:
                            s.next_token = ids[s.await_row]
                            s.await_row = -1
                            self.stats["choice_waits"] += 1
                        for s, row, src in gathered:
                            m = self._after_feed(s, ids[src])
                            if not s.done and m is not None:
                                if self._in_choice(s):  # the row just launched selected a choice token
                                    s.await_row, s.await_step = row, step_no
                                else:
                                    s.next_src = row  # its selection in the step just launched
                t3 = time.perf_counter()
                if toks:
                    prev_event, prev_buf, prev_n = event, buf, len(toks)
                    self.stats["decode_steps"] += 1
                    self._count_graphs()
                    self.stats["decode_rows"] += len(toks)
                    self.stats["generated_tokens"] += len(toks)
                gone = [s for s in active if s.done]
                active = [s for s in active if not s.done]
                for s in gone:
                    retire(s)
                t4 = time.perf_counter()
                self.stats["wait_s"] += t3 - th
                self.stats["host_s"] += (t1 - t0) + (t4 - t3) + (t2 - t1)
                self.stats["decode_s"] += (t4 - t0) - (th - t2)
                self.stats["under_s"] += th - t2
                # replies go out while the GPU computes the step just launched
                while finished:
                    s = finished.pop()
                    raw = self._finish(s, partials)
                    if raw is not None:
                        yield s.index, raw
        finally:
            if prev_event is not None:
                prev_event.synchronize()
            for h in admits:
                if h["event"] is not None:
                    h["event"].synchronize()
            for a, b in self._pf_events:  # device time of the prefills (stats only)
                self.stats["prefill_gpu_s"] += a.elapsed_time(b) * 1e-3
            self._pf_events.clear()
            if self._native is not None:
                for k, v in self._native.stats().items():
                    self.stats[k] += v
                self._native.reset_stats()
                self._native.reset()
            if P:
                self.model.clear_prefix()
            self.model.fork_defer = False
            self.model.fork_flush()
            if gc_deferred:
                _gc_defer_exit()
            clock.next()
            self.slow_iters = clock.slow


# Full-collection deferral is process-wide (gc thresholds are global) while
# several engines may run sessions at once (_threaded_stream): the first
# session to enter saves the threshold, the last to leave restores it -- a
# per-session save / restore interleaved across threads could restore a
# raised value and leave full collections deferred for the process' life.
_GC_LOCK = threading.Lock()
_GC_STATE = {"active": 0, "saved": None, "every": 0}


def _gc_defer_enter(every: int) -> None:
    with _GC_LOCK:
        if _GC_STATE["active"] == 0:
            _GC_STATE["saved"] = gc.get_threshold()
            _GC_STATE["every"] = 0
        _GC_STATE["active"] += 1
        if every > _GC_STATE["every"]:
            _GC_STATE["every"] = every
            t0, t1, t2 = _GC_STATE["saved"]
            gc.set_threshold(t0, t1, max(t2, every))


def _gc_defer_exit() -> None:
    with _GC_LOCK:
        _GC_STATE["active"] -= 1
        if _GC_STATE["active"] == 0 and _GC_STATE["saved"] is not None:
            gc.set_threshold(*_GC_STATE["saved"])
            _GC_STATE["saved"] = None
            _GC_STATE["every"] = 0


class LocalLLMBackend(EnrichmentBackend):
    """EnrichmentBackend over local engines living in THIS process (one per
    GPU; tests, smoke, single-GPU tools).  The multi-GPU service path runs one
    engine per worker process instead (:class:`ProcessLLMBackend`)."""

    name = "local"

    def __init__(self, engines: Sequence[LocalEngine], max_concurrent: int = 1) -> None:
        super().__init__(max_concurrent=max(1, len(engines)))
        self.engines = list(engines)
        self.preferred_batch_size = sum(e.cfg.max_batch for e in self.engines) * 2

    @property
    def source_tag(self) -> str:
        m = self.engines[0].model if self.engines else None
        ck = getattr(m, "checkpoint", None)
        if ck:
            return f"local:{os.path.abspath(ck)}"
        name = getattr(getattr(m, "cfg", None), "name", "echo")
        return SYNTHETIC_PREFIX + ("echo" if m is None or not hasattr(m, "cfg") else f"random-init:{name}")

    @classmethod
    def from_config(cls, cfg) -> EnrichmentBackend:
        if (cfg.local_llm_workers or "process").lower() == "process":
            return ProcessLLMBackend.from_config(cfg)
        from .workers import engine_spec, model_spec
        devices = []
        if torch.cuda.is_available():
            n = torch.cuda.device_count()
            spec = (cfg.local_llm_devices or "all").strip()
            devices = list(range(n)) if spec == "all" else [int(x) for x in spec.split(",") if x.strip()]
        if not devices:
            raise RuntimeError("LocalLLMBackend needs a ROCm GPU (torch.cuda.is_available() is False)")
        engines = []
        for d in devices:
            with torch.cuda.device(d):
                model, tok = build_model(model_spec(cfg), f"cuda:{d}")
                engines.append(LocalEngine(model, tokenizer=tok, **engine_spec(cfg)))
        return cls(engines)

    def enrich_class(self, inp: EnrichmentInput, readme: Optional[str]) -> EnrichmentResult:
        return self.enrich_batch([inp], readme)[0]

    def enrich_batch(self, inputs: Sequence[EnrichmentInput], readme: Optional[str]) -> List[EnrichmentResult]:
        out: Dict[int, EnrichmentResult] = {}
        for i, r in self.enrich_stream(inputs, readme):
            out[i] = r
        return [out[i] for i in range(len(inputs))]

    def enrich_stream(self, inputs: Iterable[EnrichmentInput], readme: Optional[str]
                      ) -> Iterator[Tuple[int, EnrichmentResult]]:
        """Every engine pulls classes from ONE shared feed as its slots free
        up (work-stealing per class: every replica gets work, however few
        classes there are); results are yielded as sequences finish."""
        src = enumerate(inputs)
        if len(self.engines) == 1:
            names: Dict[int, str] = {}

            def tagged():
                for i, inp in src:
                    names[i] = inp.full_class_name
                    yield i, inp
            eng = self.engines[0]
            with _device(eng):
                try:
                    for i, raw in eng.stream(tagged(), readme):
                        yield i, _parse(raw, names.pop(i))
                except Exception as e:  # engine failure: everything not yet returned fails
                    LOG.exception("local engine failed")
                    for i, name in list(names.items()):
                        yield i, EnrichmentResult.failure(name, f"engine failed: {e}")
                    for i, inp in src:
                        yield i, EnrichmentResult.failure(inp.full_class_name, f"engine failed: {e}")
            return
        yield from _threaded_stream(self.engines, src, readme)

    def stats(self) -> dict:
        agg: Dict[str, float] = {}
        for e in self.engines:
            for k, v in e.stats.items():
                agg[k] = agg.get(k, 0) + v
        return agg


def build_model(spec: dict, device: str):
    """(LocalLM, tokenizer) of a worker model spec: the checkpoint directory
    ``spec["path"]`` (its own tokenizer) or the random-initialised preset
    ``spec["preset"]`` (byte-level tokenizer: ``None`` = the engine default);
    ``kv_dtype`` / ``prefill_dtype`` / ``decode_dtype`` / ``max_batch`` / ``max_rows`` / ``max_seq`` override either."""
    overrides = {k: spec[k] for k in ("kv_dtype", "prefill_dtype", "decode_dtype", "max_batch", "max_rows", "max_seq") if k in spec}
    if spec.get("path"):
        from .tokenizer import load_local_model
        return load_local_model(spec["path"], device=device, **overrides)
    cfg = preset(spec.get("preset", "dmcp-coder-1b"), **overrides)
    model = LocalLM(cfg, device=device, seed=int(spec.get("seed", 0)))
    if cfg.tokenizer:
        from .tokenizer import load_asset_tokenizer
        return model, load_asset_tokenizer(cfg.tokenizer)
    return model, None


def _parse(raw: str, name: str) -> EnrichmentResult:
    return parse_enrichment_response(raw, name)


def _device(eng: LocalEngine):
    return torch.cuda.device(eng.model.device) if eng.model.device.type == "cuda" else _nullctx()


class _SharedFeed:
    """One locked iterator several engine threads take from."""

    def __init__(self, src) -> None:
        self._src = src
        self._lock = threading.Lock()
        self.done = False
        self.names: Dict[int, str] = {}

    def take(self, n: int, wait: bool = False):
        with self._lock:
            out = []
            while len(out) < n and not self.done:
                try:
                    i, inp = next(self._src)
                except StopIteration:
                    self.done = True
                    break
                self.names[i] = inp.full_class_name
                out.append((i, inp))
            return out


def _threaded_stream(engines: Sequence[LocalEngine], src, readme: Optional[str]):
    import queue
    feed = _SharedFeed(src)
    q: "queue.Queue" = queue.Queue()

    def run(eng: LocalEngine) -> None:
        try:
            with _device(eng):
                for i, raw in eng.stream(feed, readme):
                    q.put((i, raw, None))
        except BaseException as e:  # this replica stops; its taken classes fail below
            LOG.exception("local engine on %s failed", eng.model.device)
            q.put((None, None, e))
        finally:
            q.put(None)

    threads = [threading.Thread(target=run, args=(e,), name=f"engine-{k}", daemon=True)
               for k, e in enumerate(engines)]
    for t in threads:
        t.start()
    live, err = len(threads), None
    while live:
        item = q.get()
        if item is None:
            live -= 1
            continue
        i, raw, e = item
        if e is not None:
            err = e
            continue
        yield i, _parse(raw, feed.names.pop(i))
    for i, name in list(feed.names.items()):  # taken by a failed replica
        yield i, EnrichmentResult.failure(name, f"engine failed: {err}")


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


from .workers import ProcessLLMBackend  # noqa: E402  (the service's multi-GPU backend)
