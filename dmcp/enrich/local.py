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
* multi-GPU: one engine (replica) per GPU, classes sharded across replicas
  (:mod:`dmcp.parallel.replicas`) -- pure data parallelism, no collectives
  (SURVEY §5.8).
"""
from __future__ import annotations

import json
import logging
import threading
import time
from collections import deque
from dataclasses import dataclass, field
from typing import Deque, Dict, List, Optional, Sequence, Tuple

import torch

from ..models.llm import BOS, LocalLM, LMConfig, DecodeGraphs, preset
from .backend import EnrichmentBackend, build_enrichment_prompt
from .jsonfix import parse_enrichment_response
from .types import EnrichmentInput, EnrichmentResult

LOG = logging.getLogger(__name__)

QUOTE = ord('"')


def _json_safe_mask(vocab: int, with_quote: bool) -> List[int]:
    words = [0] * ((vocab + 31) // 32)
    for b in range(0x20, 0x7F):
        if b in (QUOTE, ord("\\")):
            continue
        words[b >> 5] |= 1 << (b & 31)
    if with_quote:
        words[QUOTE >> 5] |= 1 << (QUOTE & 31)
    # int32 view of the uint32 bit pattern
    return [w - (1 << 32) if w >= (1 << 31) else w for w in words]


@dataclass
class Segment:
    forced: Optional[bytes] = None   # forced bytes, or None for a free string
    min_len: int = 0
    max_len: int = 0


def build_template(inp: EnrichmentInput, desc_len=(8, 96), method_len=(6, 64), step_len=(4, 40),
                   steps: int = 2) -> List[Segment]:
    """Segments of the reply; a free segment ends with a model- or force-emitted '"'."""
    segs: List[Segment] = [Segment(b'{"description": "'), Segment(None, *desc_len),
                           Segment(b', "classTypeCorrection": null, "methods": [')]
    names = list(dict.fromkeys(inp.method_names))
    for i, name in enumerate(names):
        segs.append(Segment(b'{"methodName": ' + json.dumps(name).encode() + b', "description": "'))
        segs.append(Segment(None, *method_len))
        segs.append(Segment(b', "businessLogic": ["'))
        for s in range(steps):
            segs.append(Segment(None, *step_len))
            if s + 1 < steps:
                segs.append(Segment(b', "'))
        segs.append(Segment(b"]}" + (b", " if i + 1 < len(names) else b"")))
    segs.append(Segment(b"]}"))
    # merge adjacent forced segments
    out: List[Segment] = []
    for s in segs:
        if out and s.forced is not None and out[-1].forced is not None:
            out[-1] = Segment(out[-1].forced + s.forced)
        else:
            out.append(s)
    return out


def template_budget(segs: Sequence[Segment]) -> int:
    return sum(len(s.forced) if s.forced is not None else s.max_len + 1 for s in segs)


def fit_template(inp: EnrichmentInput, capacity: int) -> List[Segment]:
    """Largest template whose reply budget fits ``capacity`` tokens: free-string
    lengths shrink first (down to a floor), then trailing methods are dropped."""
    names = list(dict.fromkeys(inp.method_names))
    for scale in (1.0, 0.75, 0.5, 0.35, 0.25):
        def L(lo, hi):
            return (min(lo, max(2, int(hi * scale))), max(4, int(hi * scale)))
        segs = build_template(inp, L(8, 96), L(6, 64), L(4, 40))
        if template_budget(segs) <= capacity:
            return segs
    keep = len(names)
    while keep > 0:
        keep //= 2
        sub = EnrichmentInput(inp.source_code, inp.full_class_name, inp.language, inp.class_type, names[:keep])
        segs = build_template(sub, (2, 24), (2, 16), (2, 8), steps=1)
        if template_budget(segs) <= capacity:
            return segs
    return build_template(EnrichmentInput(inp.source_code, inp.full_class_name, inp.language,
                                          inp.class_type, []), (2, 16))


@dataclass
class _Seq:
    inp: EnrichmentInput
    index: int
    segs: List[Segment]
    slot: int = -1
    pos: int = 0                       # tokens already in the KV cache
    seg: int = 0
    free_len: int = 0
    forced_off: int = 0
    next_token: int = -1               # token to feed at the next decode step
    next_src: int = -1                 # ... or: row of the last launched step whose selection it is
    out: bytearray = field(default_factory=bytearray)
    done: bool = False
    prompt_tokens: int = 0
    gen_tokens: int = 0


class LocalEngine:
    """Continuous-batching, grammar-forced greedy generator over one LocalLM.

    ``jump_forward``: forced skeleton bytes are not fed one per step -- after
    a sequence's token is fed, every following token that is already decided
    (the rest of a forced segment, or the closing quote of a string at its
    length cap) is appended to the SAME step as extra rows of that sequence,
    up to ``max_rows`` rows per step.  The KV append + causal per-row
    attention of :meth:`LocalLM.decode` makes that an exact multi-token
    extend, so only free (sampled) tokens cost a step each.
    """

    MASK_NO_QUOTE, MASK_QUOTE = 0, 1
    MIN_SHARED_PREFIX = 64  # tokens; shorter common prefixes are not worth a separate prefill

    def __init__(self, model: LocalLM, use_graphs: bool = True, max_prompt_tokens: Optional[int] = None,
                 jump_forward: bool = True, shared_prefix: bool = True, pipeline: bool = True) -> None:
        self.model = model
        self.cfg: LMConfig = model.cfg
        dev = model.device
        self.masks = torch.tensor([_json_safe_mask(self.cfg.vocab_size, False),
                                   _json_safe_mask(self.cfg.vocab_size, True)], dtype=torch.int32, device=dev)
        self.graphs = DecodeGraphs(model, self.masks) if use_graphs and dev.type == "cuda" else None
        self.max_prompt_tokens = max_prompt_tokens
        self.jump_forward = jump_forward
        self.shared_prefix = shared_prefix and model.shared_prefix
        self.max_rows = model.max_rows
        self.pipeline = pipeline
        # previous step's selections for host-less gathers (graphs keep their own)
        self._last_ids = self.graphs.last_ids if self.graphs is not None else \
            torch.zeros(self.max_rows, dtype=torch.int32, device=dev)
        # pinned double buffer for the ids of the last two launched steps
        self._host_ids = [torch.zeros(self.max_rows, dtype=torch.int32, pin_memory=dev.type == "cuda")
                          for _ in range(2)]
        self.stats = {"prompt_tokens": 0, "generated_tokens": 0, "decode_steps": 0, "decode_rows": 0,
                      "prefills": 0, "decode_s": 0.0, "prefill_s": 0.0, "prefix_tokens": 0, "prefix_s": 0.0}
        self._lock = threading.Lock()

    # ---------------------------------------------------------------- api
    def generate(self, inputs: Sequence[EnrichmentInput], readme: Optional[str]) -> List[str]:
        """Returns the raw JSON reply for every input (same order)."""
        with self._lock:
            return self._generate(inputs, readme)

    # ------------------------------------------------------------ helpers
    def _prompt(self, seq: _Seq, readme: Optional[str], budget: int) -> List[int]:
        text = build_enrichment_prompt(seq.inp, readme).encode("utf-8", "replace")
        limit = self.cfg.max_seq - budget - 2
        if self.max_prompt_tokens:
            limit = min(limit, self.max_prompt_tokens)
        if limit < 16:
            raise ValueError("KV capacity too small for the reply template")
        if len(text) > limit:
            keep_tail = min(256, limit // 4)  # keep the instructions at the end
            text = text[:limit - keep_tail] + text[len(text) - keep_tail:]
        return [BOS] + list(text)

    def _select_one(self, logits: torch.Tensor, with_quote: bool) -> int:
        from .. import ops
        idx = torch.tensor([self.MASK_QUOTE if with_quote else self.MASK_NO_QUOTE], dtype=torch.int32,
                           device=logits.device)
        return int(ops.masked_argmax(logits.reshape(1, -1).contiguous(), self.masks, vocab=self.cfg.vocab_size,
                                     mask_idx=idx).item())

    def _step(self, toks: List[int], slots: List[int], poss: List[int], mrows: List[int]) -> List[int]:
        """One batched forward over the rows; returns the masked argmax of every row."""
        if self.graphs is not None:
            _, ids = self.graphs.run(toks, slots, poss, mrows)
        else:
            dev = self.model.device
            t = torch.tensor([toks, slots, poss, mrows], dtype=torch.int32, device=dev)
            _, ids = self.model.decode_select(t[0].contiguous(), t[1].contiguous(), t[2].contiguous(), self.masks,
                                              t[3].contiguous())
        return ids.cpu().tolist()

    def _advance_forced(self, s: _Seq) -> None:
        """Sets next_token from the current forced segment or finishes."""
        while s.seg < len(s.segs):
            seg = s.segs[s.seg]
            if seg.forced is None:
                return
            if s.forced_off < len(seg.forced):
                s.next_token = seg.forced[s.forced_off]
                s.forced_off += 1
                return
            s.seg += 1
            s.forced_off = 0
            s.free_len = 0
        s.done = True

    def _after_feed(self, s: _Seq, tok: int) -> Optional[bool]:
        """Grammar transition after ``tok`` entered the KV cache.  Returns None
        when the next token is already decided (``s.next_token``) or the reply
        is complete, else whether the sampled token may be the closing quote."""
        s.out.append(tok & 0xFF)
        s.pos += 1
        s.gen_tokens += 1
        seg = s.segs[s.seg] if s.seg < len(s.segs) else None
        if seg is not None and seg.forced is None:
            if tok == QUOTE:  # free string closed
                s.seg += 1
                s.forced_off = 0
                s.free_len = 0
                self._advance_forced(s)
            else:
                s.free_len += 1
                if s.free_len >= seg.max_len:
                    s.next_token = QUOTE
                    return None
                return s.free_len >= seg.min_len
        else:
            self._advance_forced(s)
        if not s.done and s.segs[s.seg].forced is None:
            return s.segs[s.seg].min_len == 0
        return None

    def _build_prompt(self, s: _Seq, readme: Optional[str]) -> List[int]:
        budget = template_budget(s.segs)
        if budget + 32 > self.cfg.max_seq:
            raise ValueError(f"reply template needs {budget} tokens > max_seq {self.cfg.max_seq}")
        return self._prompt(s, readme, budget)

    def _common_prefix(self, prompts: Sequence[List[int]]) -> int:
        """Tokens shared by the start of every prompt (instructions + README
        for classes of one project), leaving each prompt >= 1 own token."""
        if not self.shared_prefix or len(prompts) < 2:
            return 0
        first = prompts[0]
        n = min(len(p) for p in prompts) - 1
        for p in prompts[1:]:
            k = 0
            while k < n and p[k] == first[k]:
                k += 1
            n = k
            if n < self.MIN_SHARED_PREFIX:
                return 0
        return n if n >= self.MIN_SHARED_PREFIX else 0

    def _admit(self, s: _Seq, prompt: List[int], prefix: int, results: Dict[int, str],
               free_slots: List[int]) -> bool:
        """Prefill prompt + first forced segment; True if the sequence stays active.
        With a shared prefix of ``prefix`` tokens only the rest is prefilled."""
        s.slot = free_slots.pop()
        first = s.segs[0].forced or b""
        toks = prompt + list(first)
        t0 = time.perf_counter()
        start = self.model.fork_prefix(s.slot) if prefix else 0
        logits = self.model.forward_tokens(torch.tensor(toks[start:], dtype=torch.int32), s.slot, start)
        self.stats["prefill_s"] += time.perf_counter() - t0
        self.stats["prefills"] += 1
        self.stats["prompt_tokens"] += len(toks) - start
        s.prompt_tokens = len(prompt)
        s.out.extend(first)
        s.pos = len(toks)
        s.seg, s.forced_off = 1, 0
        if s.seg < len(s.segs) and s.segs[s.seg].forced is None:
            s.next_token = self._select_one(logits, s.segs[s.seg].min_len == 0)
        else:
            self._advance_forced(s)
        if s.done:
            results[s.index] = s.out.decode("utf-8", "replace")
            free_slots.append(s.slot)
            return False
        return True

    def _generate(self, inputs: Sequence[EnrichmentInput], readme: Optional[str]) -> List[str]:
        cfg = self.cfg
        reply_cap = cfg.max_seq - max(64, cfg.max_seq // 4)
        results: Dict[int, str] = {}
        prompts: Dict[int, List[int]] = {}
        pending: Deque[_Seq] = deque()
        for i, inp in enumerate(inputs):
            s = _Seq(inp, i, fit_template(inp, reply_cap))
            try:
                prompts[i] = self._build_prompt(s, readme)
                pending.append(s)
            except Exception as e:
                results[i] = json.dumps({"error": str(e)})
        # one prefill of the common prefix (instructions + README) for all
        prefix = self._common_prefix(list(prompts.values()))
        if prefix:
            t0 = time.perf_counter()
            self.model.set_prefix(prompts[pending[0].index][:prefix])
            self.stats["prefix_s"] += time.perf_counter() - t0
            self.stats["prefix_tokens"] += prefix
        try:
            if self.pipeline:
                self._run_pipelined(pending, prompts, prefix, results)
            else:
                self._run(pending, prompts, prefix, results)
        finally:
            if prefix:
                self.model.clear_prefix()
        return [results[i] for i in range(len(inputs))]

    def _run(self, pending: Deque[_Seq], prompts: Dict[int, List[int]], prefix: int,
             results: Dict[int, str]) -> None:
        cfg = self.cfg
        free_slots = list(range(cfg.max_batch - 1, -1, -1))
        active: List[_Seq] = []
        while pending or active:
            while pending and free_slots:
                s = pending.popleft()
                if self._admit(s, prompts.pop(s.index), prefix, results, free_slots):
                    active.append(s)
            if not active:
                continue
            # one batched step: every active sequence feeds its next token, plus
            # (jump-forward) every already-decided token after it
            t0 = time.perf_counter()
            toks: List[int] = []
            slots: List[int] = []
            poss: List[int] = []
            mrows: List[int] = []
            sample_at: List[Tuple[_Seq, int]] = []
            spare = self.max_rows - len(active)  # rows beyond one per sequence
            for s in active:
                tok = s.next_token
                while True:
                    toks.append(tok)
                    slots.append(s.slot)
                    poss.append(s.pos)
                    mrows.append(self.MASK_NO_QUOTE)
                    q = self._after_feed(s, tok)
                    if s.done:
                        break
                    if q is not None:  # the next token is sampled from this row's logits
                        mrows[-1] = self.MASK_QUOTE if q else self.MASK_NO_QUOTE
                        sample_at.append((s, len(toks) - 1))
                        break
                    if not self.jump_forward or spare <= 0:
                        break  # decided token waits for the next step
                    spare -= 1
                    tok = s.next_token
            ids = self._step(toks, slots, poss, mrows)
            for s, r in sample_at:
                s.next_token = ids[r]
            self.stats["decode_s"] += time.perf_counter() - t0
            self.stats["decode_steps"] += 1
            self.stats["decode_rows"] += len(toks)
            self.stats["generated_tokens"] += len(toks)
            still = []
            for s in active:
                if s.done:
                    results[s.index] = s.out.decode("utf-8", "replace")
                    free_slots.append(s.slot)
                else:
                    still.append(s)
            active = still


    # ------------------------------------------------------ pipelined loop
    def _launch(self, toks: List[int], slots: List[int], poss: List[int], mrows: List[int],
                srcs: List[int], buf: int):
        """Launches one step; enqueues the copy of its ids to pinned buffer
        ``buf``; returns the event that completes with that copy."""
        if self.graphs is not None:
            _, ids = self.graphs.run(toks, slots, poss, mrows, srcs)
        else:
            dev = self.model.device
            t = torch.tensor([toks, slots, poss, mrows, srcs], dtype=torch.int32, device=dev)
            _, ids = self.model.decode_select_gather(t[0].contiguous(), t[4].contiguous(), self._last_ids,
                                                     t[1].contiguous(), t[2].contiguous(), self.masks,
                                                     t[3].contiguous())
        n = len(toks)
        host = self._host_ids[buf]
        host[:n].copy_(ids[:n], non_blocking=self.model.device.type == "cuda")
        if self.model.device.type == "cuda":
            ev = torch.cuda.Event()
            ev.record()
            return ev
        return None

    def _speculative_mask(self, s: _Seq) -> int:
        """Mask row for a row whose token is still on the device (a free-text
        selection): the state after feeding any token but the closing quote
        -- the only case in which this row's own selection is used."""
        seg = s.segs[s.seg]
        return self.MASK_QUOTE if s.free_len + 1 >= seg.min_len else self.MASK_NO_QUOTE

    def _run_pipelined(self, pending: Deque[_Seq], prompts: Dict[int, List[int]], prefix: int,
                       results: Dict[int, str]) -> None:
        """Continuous batching with the host one step behind the device.

        Each iteration builds step k's rows from the state known after
        step k-1's inputs: a sequence whose next token is step k-1's
        selection gets ONE gathered row (its mask row assumes the token is
        not the closing quote -- if it is, that row's own selection is simply
        not used); every other sequence gets its literal token and, with
        jump-forward, the decided tokens after it.  Step k is launched, and
        only then does the host wait for step k-1's ids and run the grammar
        transitions of step k's gathered rows -- while the GPU computes
        step k.  The price: forced bytes that follow a sampled closing quote
        start one step later than in :meth:`_run`."""
        cfg = self.cfg
        free_slots = list(range(cfg.max_batch - 1, -1, -1))
        active: List[_Seq] = []
        prev_event = None
        prev_buf = 1
        while pending or active:
            while pending and free_slots:
                s = pending.popleft()
                if self._admit(s, prompts.pop(s.index), prefix, results, free_slots):
                    active.append(s)
            if not active:
                continue
            t0 = time.perf_counter()
            toks: List[int] = []
            slots: List[int] = []
            poss: List[int] = []
            mrows: List[int] = []
            srcs: List[int] = []
            gathered: List[Tuple[_Seq, int, int]] = []  # (seq, row, source row of the previous step)
            spare = self.max_rows - len(active)
            for s in active:
                if s.next_src >= 0:
                    gathered.append((s, len(toks), s.next_src))
                    toks.append(0)
                    slots.append(s.slot)
                    poss.append(s.pos)
                    mrows.append(self._speculative_mask(s))
                    srcs.append(s.next_src)
                    s.next_src = -1
                    continue
                tok = s.next_token
                while True:
                    toks.append(tok)
                    slots.append(s.slot)
                    poss.append(s.pos)
                    mrows.append(self.MASK_NO_QUOTE)
                    srcs.append(-1)
                    q = self._after_feed(s, tok)
                    if s.done:
                        break
                    if q is not None:  # this row's selection is the next token
                        mrows[-1] = self.MASK_QUOTE if q else self.MASK_NO_QUOTE
                        s.next_src = len(toks) - 1
                        break
                    if not self.jump_forward or spare <= 0:
                        break
                    spare -= 1
                    tok = s.next_token
            buf = 1 - prev_buf
            event = self._launch(toks, slots, poss, mrows, srcs, buf)
            # the previous step's ids: the tokens this step's gathered rows fed
            if gathered:
                if prev_event is not None:
                    prev_event.synchronize()
                ids = self._host_ids[prev_buf]
                for s, row, src in gathered:
                    q = self._after_feed(s, int(ids[src]))
                    if not s.done and q is not None:
                        s.next_src = row  # its selection in the step just launched
            prev_event, prev_buf = event, buf
            self.stats["decode_s"] += time.perf_counter() - t0
            self.stats["decode_steps"] += 1
            self.stats["decode_rows"] += len(toks)
            self.stats["generated_tokens"] += len(toks)
            still = []
            for s in active:
                if s.done:
                    results[s.index] = s.out.decode("utf-8", "replace")
                    free_slots.append(s.slot)
                else:
                    still.append(s)
            active = still
        if prev_event is not None:
            prev_event.synchronize()


class LocalLLMBackend(EnrichmentBackend):
    """EnrichmentBackend over one or more local engines (one per GPU)."""

    name = "local"

    def __init__(self, engines: Sequence[LocalEngine], max_concurrent: int = 1) -> None:
        super().__init__(max_concurrent=max(1, len(engines)))
        self.engines = list(engines)
        self.preferred_batch_size = sum(e.cfg.max_batch for e in self.engines) * 2

    @classmethod
    def from_config(cls, cfg) -> "LocalLLMBackend":
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
                model = LocalLM(preset(cfg.local_llm_preset, kv_dtype=cfg.local_llm_kv_dtype), device=f"cuda:{d}",
                                seed=0)
                engines.append(LocalEngine(model))
        return cls(engines)

    def enrich_class(self, inp: EnrichmentInput, readme: Optional[str]) -> EnrichmentResult:
        return self.enrich_batch([inp], readme)[0]

    def enrich_batch(self, inputs: Sequence[EnrichmentInput], readme: Optional[str]) -> List[EnrichmentResult]:
        if not inputs:
            return []
        from ..parallel.replicas import ReplicaPool
        n, E = len(inputs), len(self.engines)
        # one engine: everything in one continuous batch; several: work-stealing
        # chunks big enough to keep each replica's batch full
        chunk = n if E == 1 else max(2 * max(e.cfg.max_batch for e in self.engines), -(-n // (2 * E)))
        pool = ReplicaPool(self.engines, chunk_for=lambda e: chunk)

        def ctx(eng):
            return torch.cuda.device(eng.model.device) if eng.model.device.type == "cuda" else _nullctx()

        raw = pool.map(lambda eng, items: eng.generate(items, readme), list(inputs), device_ctx=ctx)
        results = []
        for inp, r in zip(inputs, raw):
            if isinstance(r, BaseException) or r is None:
                results.append(EnrichmentResult.failure(inp.full_class_name, str(r) if r is not None else "no output"))
            else:
                results.append(parse_enrichment_response(r, inp.full_class_name))
        return results

    def stats(self) -> dict:
        agg: Dict[str, float] = {}
        for e in self.engines:
            for k, v in e.stats.items():
                agg[k] = agg.get(k, 0) + v
        return agg


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
