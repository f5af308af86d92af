"""One worker process per GPU for the local enrichment model -- MI355X extension.

Enrichment requests are independent (one prompt per class,
``ClaudeApiClient.java:288-329``; the reference runs one virtual thread per
class behind a semaphore, ``:354-388``), so multi-GPU scaling is pure data
parallelism: every MI355X holds a full copy of the model and
its own KV-cache slab, and classes are dealt out by ONE pool in the parent.
Each replica lives in its own process:

* the parent (REST / MCP / CLI service) starts the workers before it touches
  HIP and never initialises the GPU itself -- each child sees exactly one
  device (``HIP_VISIBLE_DEVICES``), so a fault or hang on one GPU kills one
  child, never the server;
* each engine's host work per decode step (grammar state machine, row
  packing) runs on its own interpreter -- N replicas driven by N threads of
  one process would serialise on the GIL;
* parent and child talk over the child's stdin / stdout: length-prefixed
  JSON frames (``begin`` readme / ``items`` / ``end`` down; ``ready`` /
  ``result`` / ``done`` / ``error`` up); the child's logs go to stderr;
* a child runs ONE engine stream over all the sessions it was dealt
  (:class:`dmcp.enrich.feeds.MultiFeed`): two projects on one GPU share its
  continuous batch instead of queueing one behind the other.

Dealing (:class:`GpuWorkerPool`):

* several streams (projects: concurrent REST requests, the sync scheduler,
  bulk indexing) run at once.  Each live worker is OWNED by one stream at a
  time -- the workers are split evenly over the streams that still have
  classes to deal, in arrival order -- so new classes go where their
  project's shared prompt prefix is resident; a worker handed to another
  stream keeps decoding what it holds of the first next to the new work;
* within a stream the pending classes are dealt ``ceil(pending / owned)``
  per worker (capped at ``capacity`` in flight), topped up as replies return:
  a 257-class project on 8 GPUs is 32-33 classes per GPU, not 257 on GPU 0;
* a worker that dies (EOF on its pipe, a non-zero exit, or no frame for
  ``hang_timeout_s`` while it holds work -- then it is killed) fails the
  classes it held (Phase 3 retries them); the rest go to the live workers.
  A dead worker is replaced by a FRESH child at the next stream; a
  GPU-touched process is never restarted in place.
"""
from __future__ import annotations

import json
import logging
import operator
import os
import queue
import struct
import subprocess
import sys
import threading
import time
from typing import Any, Dict, Iterable, Iterator, List, Optional, Sequence, Tuple

from .backend import SYNTHETIC_PREFIX, EnrichmentBackend
from .jsonfix import parse_enrichment_response
from .types import EnrichmentInput, EnrichmentResult

LOG = logging.getLogger(__name__)

_HDR = struct.Struct("<I")
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def send_frame(stream, obj) -> None:
    data = json.dumps(obj, separators=(",", ":")).encode("utf-8")
    stream.write(_HDR.pack(len(data)) + data)
    stream.flush()


def recv_frame(stream) -> Optional[dict]:
    hdr = stream.read(_HDR.size)
    if len(hdr) < _HDR.size:
        return None
    n = _HDR.unpack(hdr)[0]
    data = stream.read(n)
    if len(data) < n:
        return None
    return json.loads(data.decode("utf-8"))


def _inp_to_wire(inp: EnrichmentInput) -> list:
    return [inp.source_code, inp.full_class_name, inp.language, inp.class_type, list(inp.method_names)]


def _inp_from_wire(v: list) -> EnrichmentInput:
    return EnrichmentInput(v[0], v[1], v[2], v[3], list(v[4]))


def visible_gpus() -> int:
    """GPUs on this host without initialising HIP in this process
    (``torch.cuda.device_count`` does not create a context on this image)."""
    try:
        import torch
        return int(torch.cuda.device_count())
    except Exception:
        return 0


# ------------------------------------------------------------------ parent
class _Worker:
    def __init__(self, index: int, device: str, pool: "GpuWorkerPool", env_extra: Optional[dict] = None) -> None:
        self.index = index
        self.device = device  # "cuda:<physical id>" or "cpu"
        self.pool = pool
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        env["PYTHONPATH"] = ROOT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        if device.startswith("cuda"):
            phys = device.split(":", 1)[1] if ":" in device else "0"
            env["HIP_VISIBLE_DEVICES"] = phys
            env.pop("CUDA_VISIBLE_DEVICES", None)
            env.pop("ROCR_VISIBLE_DEVICES", None)
        env.update(env_extra or {})
        self.proc = subprocess.Popen([sys.executable, "-u", "-m", "dmcp.enrich.workers"], stdin=subprocess.PIPE,
                                     stdout=subprocess.PIPE, stderr=None, env=env, cwd=ROOT)
        self.alive = True
        self.closing = False
        self.ready = False
        self.info: dict = {}
        self.inflight: Dict[int, Dict[int, str]] = {}  # stream id -> key -> class name
        self.owner: Optional["_Stream"] = None
        self.last_frame = time.monotonic()  # last sign of progress (frame, or work handed to an idle worker)
        self.stats: Dict[str, float] = {}
        self.sent = 0
        self._wlock = threading.Lock()
        self._reader = threading.Thread(target=self._read, name=f"gpu-worker-{index}-rx", daemon=True)
        self._reader.start()

    def held(self) -> int:
        return sum(len(d) for d in self.inflight.values())

    def _read(self) -> None:
        out = self.proc.stdout
        while True:
            try:
                msg = recv_frame(out)
            except Exception as e:  # corrupt frame: treat as death
                LOG.error("worker %d: bad frame: %s", self.index, e)
                msg = None
            # routed with this worker object, not its index: a replaced
            # worker's late EOF must not mark its successor dead
            self.pool._on_frame(self, msg)
            if msg is None:
                return

    def send(self, obj) -> bool:
        if not self.alive:
            return False
        try:
            with self._wlock:
                send_frame(self.proc.stdin, obj)
            return True
        except (BrokenPipeError, OSError, ValueError):
            return False

    def kill(self) -> None:
        self.alive = False
        try:
            self.proc.kill()
        except Exception:
            pass

    def close(self, timeout: float = 30.0) -> None:
        self.closing = True
        if self.proc.poll() is None:
            self.send({"op": "shutdown"})
            try:
                self.proc.stdin.close()
            except Exception:
                pass
            try:
                self.proc.wait(timeout=timeout)
            except subprocess.TimeoutExpired:
                self.proc.kill()
                self.proc.wait()
        self.alive = False


class _Stream:
    """One enrichment stream (one project's pending classes) in the pool."""

    def __init__(self, sid: int, readme: Optional[str], inputs: Iterable[EnrichmentInput]) -> None:
        self.sid = sid
        self.readme = readme
        self.hint = operator.length_hint(inputs, -1)  # pending classes, when the caller knows them
        self.src = enumerate(inputs)
        self.taken = 0
        self.exhausted = False
        self.events: "queue.Queue" = queue.Queue()
        self.begun: List[_Worker] = []      # workers that got this stream's ``begin``
        self.ended: set = set()             # ... and its ``end``
        self.finished: set = set()          # ... and answered ``done``
        self.stats: Dict[str, float] = {}
        self.items_per_worker: Dict[int, int] = {}

    def remaining(self) -> Optional[int]:
        return None if self.hint < 0 else max(0, self.hint - self.taken)


class GpuWorkerPool:
    """N worker processes, one per device, shared by every enrichment stream
    of the service (:meth:`stream` may run in several threads at once).
    Spawn (cheap: the children import nothing heavy until ``init``) before
    this process touches HIP."""

    def __init__(self, devices: Sequence[str], model: dict, engine: Optional[dict] = None,
                 hang_timeout_s: float = 300.0, start_timeout_s: float = 900.0, env_extra: Optional[dict] = None,
                 init: bool = True) -> None:
        if not devices:
            raise ValueError("GpuWorkerPool needs at least one device")
        self.devices = list(devices)
        self.model = dict(model)
        self.engine = dict(engine or {})
        self.hang_timeout_s = hang_timeout_s
        self.start_timeout_s = start_timeout_s
        self.env_extra = env_extra
        self.control: "queue.Queue" = queue.Queue()  # ready / init errors
        self._lock = threading.RLock()               # worker ownership, in-flight maps, streams
        self._init_lock = threading.Lock()           # one (re)spawn + init at a time
        self.streams: Dict[int, _Stream] = {}        # arrival order
        self.workers: List[_Worker] = [self._spawn(i) for i in range(len(self.devices))]
        self.sid = 0
        self.deaths = 0
        self.per_worker_items: Dict[int, int] = {}
        self._initialised = False
        if init:
            self.init()

    def _spawn(self, i: int) -> _Worker:
        extra = dict(self.env_extra or {})
        if self.devices[i] == "cpu" and "OMP_NUM_THREADS" not in extra:
            # CPU rehearsal: share the cores (oversubscribed OpenMP spin-waits
            # make every worker crawl)
            try:
                cpus = len(os.sched_getaffinity(0))
            except (AttributeError, OSError):
                cpus = os.cpu_count() or 1
            n_cpu = sum(1 for d in self.devices if d == "cpu")
            extra["OMP_NUM_THREADS"] = str(max(1, cpus // max(1, n_cpu)))
        return _Worker(i, self.devices[i], self, extra)

    @property
    def capacity(self) -> int:
        """Classes in flight per worker: its KV slots plus a look-ahead, so
        the continuous batch never drains while replies travel."""
        mb = int(self.model.get("max_batch", 256))
        return mb + max(2, mb // 2)

    # ------------------------------------------------------------ frames
    def _current(self, w: "_Worker") -> bool:
        """False for frames of a worker that was already replaced."""
        return 0 <= w.index < len(self.workers) and self.workers[w.index] is w

    def _on_frame(self, w: _Worker, msg: Optional[dict]) -> None:
        """Reader-thread entry: routes one frame (None = EOF) of ``w``."""
        if not self._current(w):
            return
        if msg is None:
            with self._lock:
                if w.alive and not w.closing:
                    LOG.error("worker %d on %s exited (rc=%s) holding %d classes", w.index, w.device,
                              w.proc.poll(), w.held())
                w.alive = False
                self._rebalance()
            self.control.put((w, None))
            self._wake_all(("dead", w))
            return
        w.last_frame = time.monotonic()
        op = msg.get("op")
        if op in ("result", "done"):
            s = self.streams.get(msg.get("sid"))
            if s is not None:
                s.events.put((w, msg))
            elif op == "result":  # a finished / abandoned stream's late reply: only the bookkeeping
                with self._lock:
                    d = w.inflight.get(msg.get("sid"))
                    if d is not None:
                        for k, _ in msg["items"]:
                            d.pop(k, None)
                        if not d:
                            w.inflight.pop(msg.get("sid"), None)
            return
        if op == "error":
            LOG.error("worker %d on %s: %s", w.index, w.device, msg.get("msg"))
            with self._lock:
                w.kill()  # it exits on its own; never reused
                self._rebalance()
            self._wake_all(("dead", w))
        self.control.put((w, msg))

    def _wake_all(self, ev) -> None:
        for s in list(self.streams.values()):
            s.events.put(ev)

    # ------------------------------------------------------------ life cycle
    def init(self) -> None:
        """Builds the model in every worker not yet ready (in parallel) and
        waits for all of them."""
        with self._init_lock:
            self._init_locked()

    def _init_locked(self) -> None:
        for w in self.workers:
            if w.alive and not w.ready:
                w.send({"op": "init", "model": self.model, "engine": self.engine,
                        "device": "cpu" if w.device == "cpu" else "cuda:0"})
        deadline = time.monotonic() + self.start_timeout_s
        while any(w.alive and not w.ready for w in self.workers):
            left = deadline - time.monotonic()
            if left <= 0:
                for w in self.workers:
                    if not w.ready:
                        LOG.error("worker %d on %s did not start in %.0f s", w.index, w.device, self.start_timeout_s)
                        w.kill()
                break
            try:
                who, msg = self.control.get(timeout=min(1.0, left))
            except queue.Empty:
                continue
            if msg is not None and msg.get("op") == "ready" and self._current(who):
                with self._lock:
                    who.ready = True
                    who.info = msg
                    self._rebalance()
                LOG.info("GPU worker %d ready on %s (pid %s)", who.index, who.device, msg.get("pid"))
        if not any(w.ready and w.alive for w in self.workers):
            raise RuntimeError("no GPU worker started")
        self._initialised = True

    def _replace_dead(self) -> None:
        """Dead workers are replaced by fresh children (never restarted in
        place); the new ones load the model while running streams go on."""
        with self._init_lock:
            respawned = False
            with self._lock:
                for i, w in enumerate(self.workers):
                    if not w.alive:
                        w.kill()
                        self.workers[i] = self._spawn(i)
                        respawned = True
            if respawned:
                self._init_locked()

    def live(self) -> List[_Worker]:
        return [w for w in self.workers if w.alive and w.ready]

    # ------------------------------------------------------------ dealing
    def _rebalance(self) -> None:
        """Splits the live workers over the streams that still have classes
        to deal (arrival order; the first ``n % k`` get one more), keeping
        current owners where the split allows.  Caller holds ``_lock``."""
        live = self.live()
        wanting = [s for s in self.streams.values() if not s.exhausted]
        quota: Dict[int, int] = {}
        if wanting:
            n, k = len(live), len(wanting)
            for j, s in enumerate(wanting):
                quota[s.sid] = n // k + (1 if j < n % k else 0)
        kept: Dict[int, int] = {}
        free: List[_Worker] = []
        for w in live:
            o = w.owner
            if o is not None and o.sid in quota and kept.get(o.sid, 0) < quota[o.sid]:
                kept[o.sid] = kept.get(o.sid, 0) + 1
            else:
                free.append(w)
        # a free worker goes to the stream lacking the most; prefer workers
        # that hold nothing, so no stream waits behind another's session
        free.sort(key=lambda w: (w.held(), w.index))
        for w in free:
            lacking = [s for s in wanting if kept.get(s.sid, 0) < quota[s.sid]]
            new = lacking[0] if lacking else None
            self._assign(w, new)
            if new is not None:
                kept[new.sid] = kept.get(new.sid, 0) + 1
        for w in self.workers:
            if not (w.alive and w.ready):
                w.owner = None

    def _assign(self, w: _Worker, s: Optional[_Stream]) -> None:
        old = w.owner
        if old is s:
            return
        if old is not None and w in old.begun and w not in old.ended:
            old.ended.add(w)  # it finishes what it holds of ``old``, then serves ``s``
            w.send({"op": "end", "sid": old.sid})
            old.events.put(("wake", w))
        w.owner = s
        if s is not None:
            s.events.put(("wake", w))

    def _top_up(self, s: _Stream) -> List[Tuple[int, Any]]:
        """Begins ``s`` on the workers it owns and deals them its pending
        classes (``ceil(pending / owned)`` each, at most ``capacity`` in
        flight).  Returns failures to yield.  Caller holds ``_lock``."""
        owned = [w for w in self.workers if w.owner is s and w.alive and w.ready]
        fails: List[Tuple[int, Any]] = []
        for w in owned:
            if w not in s.begun:
                s.begun.append(w)
                if not w.send({"op": "begin", "sid": s.sid, "readme": s.readme}):
                    w.alive = False
        owned = [w for w in owned if w.alive]
        if s.exhausted or not owned:
            return fails
        cap = self.capacity
        rem = s.remaining()
        if rem == 0:  # the caller's hint is used up but its iterator is not: deal by capacity
            rem = None
        held = [len(w.inflight.get(s.sid, ())) for w in owned]
        if rem is None:
            targets = [cap] * len(owned)
        else:
            q, r = divmod(rem + sum(held), len(owned))
            # the +1 shares go to the workers already holding the most, so a
            # top-up never moves work that is already balanced
            order = sorted(range(len(owned)), key=lambda i: (-held[i], owned[i].index))
            targets = [0] * len(owned)
            for rank, i in enumerate(order):
                targets[i] = min(cap, q + (1 if rank < r else 0))
        chunk_min = max(1, cap // 8)
        for w, h, t in zip(owned, held, targets):
            need = t - h
            if need <= 0 or (h and need < min(chunk_min, t // 2 or 1)):
                continue
            items = []
            d = w.inflight.setdefault(s.sid, {})
            while len(items) < need:
                try:
                    i, inp = next(s.src)
                except StopIteration:
                    s.exhausted = True
                    break
                s.taken += 1
                items.append([i, _inp_to_wire(inp)])
                d[i] = inp.full_class_name
            if items:
                if w.held() == len(items):  # an idle worker gets work: its hang clock starts now
                    w.last_frame = time.monotonic()
                self.per_worker_items[w.index] = self.per_worker_items.get(w.index, 0) + len(items)
                s.items_per_worker[w.index] = s.items_per_worker.get(w.index, 0) + len(items)
                w.sent += len(items)
                if not w.send({"op": "items", "sid": s.sid, "items": items}):
                    w.alive = False
            if not d:
                w.inflight.pop(s.sid, None)
            if s.exhausted:
                break
        if s.exhausted:
            self._rebalance()  # its workers may serve other streams once they drain it
        return fails

    def _fail_dead(self, s: _Stream) -> List[Tuple[int, Any]]:
        out: List[Tuple[int, Any]] = []
        for w in self.workers + [w for w in s.begun if w not in self.workers]:
            if not w.alive and s.sid in w.inflight:
                self.deaths += 1
                for k in w.inflight.pop(s.sid):
                    out.append((k, RuntimeError(f"GPU worker died (worker {w.index} on {w.device})")))
        return out

    def _complete(self, s: _Stream) -> bool:
        if not s.exhausted:
            return False
        if any(s.sid in w.inflight for w in s.begun):
            return False
        return all(w in s.finished or not w.alive for w in s.begun)

    def stream(self, inputs: Iterable[EnrichmentInput], readme: Optional[str]
               ) -> Iterator[Tuple[int, Any]]:
        """Yields ``(input index, raw reply str | Exception)`` as replies
        arrive, from whichever worker finished them.  Safe to run from
        several threads at once (one stream per project).  A caller that
        stops early still ends its session in every worker: each finishes
        what it was sent (late replies are dropped) and serves the next."""
        self._replace_dead()
        with self._lock:
            self.sid += 1
            s = _Stream(self.sid, readme, inputs)
            self.streams[s.sid] = s
            self._rebalance()
        try:
            yield from self._run(s)
        finally:
            with self._lock:
                for w in s.begun:
                    if w not in s.ended and w.alive:
                        s.ended.add(w)
                        w.send({"op": "end", "sid": s.sid})
                s.exhausted = True
                self.streams.pop(s.sid, None)
                for w in self.workers:
                    if w.owner is s:
                        w.owner = None
                self._rebalance()

    def _run(self, s: _Stream) -> Iterator[Tuple[int, Any]]:
        while True:
            with self._lock:
                out = self._fail_dead(s)
                out += self._top_up(s)
                for w in s.begun:  # dealt out: close the sessions so the engines drain
                    if s.exhausted and w not in s.ended and w.alive:
                        s.ended.add(w)
                        w.send({"op": "end", "sid": s.sid})
                starved = not self.live() and not s.exhausted
                if starved:
                    for i, inp in s.src:  # nothing can run the rest: every remaining class fails
                        out.append((i, RuntimeError("no live GPU worker")))
                    s.exhausted = True
                    out += self._fail_dead(s)
                done = self._complete(s)
            yield from out
            if done:
                return
            try:
                ev = s.events.get(timeout=1.0)
            except queue.Empty:
                now = time.monotonic()
                with self._lock:
                    for w in s.begun:
                        if w.alive and w.inflight.get(s.sid) and now - w.last_frame > self.hang_timeout_s:
                            LOG.error("worker %d on %s sent nothing for %.0f s with %d classes: killing it",
                                      w.index, w.device, self.hang_timeout_s, w.held())
                            w.kill()
                            self._rebalance()
                continue
            w, msg = ev
            if not isinstance(msg, dict):
                continue  # a wake-up: ownership or liveness changed
            out = []
            with self._lock:
                if msg["op"] == "result":
                    d = w.inflight.get(s.sid, {})
                    for k, raw in msg["items"]:
                        if d.pop(k, None) is not None:
                            out.append((k, raw))
                    if not d:
                        w.inflight.pop(s.sid, None)
                elif msg["op"] == "done":
                    w.stats = msg.get("stats") or {}
                    for k, v in w.stats.items():
                        if isinstance(v, (int, float)):
                            s.stats[k] = s.stats.get(k, 0) + v
                    s.finished.add(w)
            yield from out

    def stats(self) -> dict:
        agg: Dict[str, float] = {}
        for w in self.workers:
            for k, v in (w.stats or {}).items():
                if isinstance(v, (int, float)):
                    agg[k] = agg.get(k, 0) + v
        agg["workers"] = len(self.workers)
        agg["worker_deaths"] = self.deaths
        return agg

    def close(self) -> None:
        for w in self.workers:
            w.close()


class ProcessLLMBackend(EnrichmentBackend):
    """The service's local-model backend: a :class:`GpuWorkerPool` (one
    process per GPU) behind the :class:`EnrichmentBackend` contract.  One
    instance serves every caller of the service (REST requests, the sync
    scheduler, bulk indexing threads) concurrently."""

    name = "local"

    def __init__(self, pool: GpuWorkerPool) -> None:
        super().__init__(max_concurrent=1)
        self.pool = pool
        self.preferred_batch_size = pool.capacity * len(pool.workers)

    @property
    def source_tag(self) -> str:
        spec = getattr(self.pool, "model", None) or {}
        if spec.get("path"):
            return f"local:{os.path.abspath(spec['path'])}"
        p = spec.get("preset", "dmcp-coder-1b")
        return SYNTHETIC_PREFIX + ("echo" if p == "echo" else f"random-init:{p}")

    @classmethod
    def from_config(cls, cfg, devices: Optional[Sequence[str]] = None) -> "ProcessLLMBackend":
        if devices is None:
            devices = worker_devices(cfg.local_llm_devices)
        return cls(GpuWorkerPool(devices, model_spec(cfg), engine=engine_spec(cfg)))

    def enrich_class(self, inp: EnrichmentInput, readme: Optional[str]) -> EnrichmentResult:
        return self.enrich_batch([inp], readme)[0]

    def enrich_batch(self, inputs: Sequence[EnrichmentInput], readme: Optional[str]) -> List[EnrichmentResult]:
        out: Dict[int, EnrichmentResult] = {}
        for i, r in self.enrich_stream(inputs, readme):
            out[i] = r
        return [out[i] for i in range(len(inputs))]

    def enrich_stream(self, inputs: Iterable[EnrichmentInput], readme: Optional[str]
                      ) -> Iterator[Tuple[int, EnrichmentResult]]:
        names: Dict[int, str] = {}
        for i, raw in self.pool.stream(_Tagged(inputs, names), readme):
            name = names.pop(i, "?")
            if isinstance(raw, BaseException):
                yield i, EnrichmentResult.failure(name, str(raw))
            else:
                yield i, parse_enrichment_response(raw, name)

    def stats(self) -> dict:
        return self.pool.stats()

    def close(self) -> None:
        self.pool.close()
        super().close()


class _Tagged:
    """The caller's inputs, recording each one's class name by index as it
    is taken; keeps the caller's length hint for the pool's dealing."""

    def __init__(self, inputs: Iterable[EnrichmentInput], names: Dict[int, str]) -> None:
        self.inputs = inputs
        self.names = names

    def __length_hint__(self):
        h = operator.length_hint(self.inputs, -1)
        return h if h >= 0 else NotImplemented

    def __iter__(self):
        for i, inp in enumerate(self.inputs):
            self.names[i] = inp.full_class_name
            yield inp


def worker_devices(spec: str) -> List[str]:
    """Worker devices of ``LOCAL_LLM_DEVICES``: ``all`` (every visible GPU),
    a comma list of GPU ids, or ``cpu`` entries (a CPU rehearsal worker each;
    tests and hosts without a GPU)."""
    spec = (spec or "all").strip()
    if spec == "all":
        devices = [f"cuda:{d}" for d in range(visible_gpus())]
    else:
        devices = ["cpu" if x.strip() == "cpu" else f"cuda:{int(x)}" for x in spec.split(",") if x.strip()]
    if not devices:
        raise RuntimeError("the local enrichment backend needs a ROCm GPU (none visible)")
    return devices


def model_spec(cfg) -> dict:
    """The worker model spec of a :class:`dmcp.config.Config`."""
    mb = int(cfg.local_llm_max_batch)
    spec = {"preset": cfg.local_llm_preset, "kv_dtype": cfg.local_llm_kv_dtype, "max_batch": mb,
            # rows per decode step: 1.5 x the slots (jump-forward rows), within
            # the hand-written decode GEMMs' 1,024 (TGEMM_MAX_ROWS)
            "max_rows": max(mb, min(1024, max(256, mb * 3 // 2))), "seed": 0,
            "prefill_dtype": getattr(cfg, "local_llm_prefill_dtype", "auto"),
            "decode_dtype": getattr(cfg, "local_llm_decode_dtype", "bf16")}
    if getattr(cfg, "local_llm_model_path", ""):
        spec["path"] = cfg.local_llm_model_path
    return spec


def engine_spec(cfg) -> dict:
    """LocalEngine keyword arguments of a :class:`dmcp.config.Config`."""
    return {"max_new_tokens": int(cfg.local_llm_max_new_tokens),
            "fork_methods": bool(getattr(cfg, "local_llm_fork_methods", True)),
            "fork_max_context": int(getattr(cfg, "local_llm_fork_max_context", 0)),
            "reply_shape": {"desc": int(getattr(cfg, "local_llm_desc_max_bytes", 0)),
                            "method": int(getattr(cfg, "local_llm_method_max_bytes", 0)),
                            "step": int(getattr(cfg, "local_llm_step_max_bytes", 0)),
                            "max_steps": int(getattr(cfg, "local_llm_max_steps", 0))}}


# ------------------------------------------------------------------ child
class _EchoEngine:
    """``preset: "echo"`` -- a model-free engine for rehearsing the pool on
    the CPU: a continuous batch in which every class takes ``steps`` steps
    of ``step_s`` seconds (latency-bound, like the GPU engine at these batch
    sizes) and is answered with a grammar-shaped reply."""

    def __init__(self, step_s: float = 0.05, max_batch: int = 512, steps: int = 1) -> None:
        self.step_s = step_s
        self.steps = max(1, steps)
        self.max_batch = max_batch
        self.stats: Dict[str, float] = {"decode_steps": 0, "prefills": 0}

    def stream(self, feed, readme):
        active: List[list] = []  # [steps left, key, input]
        while True:
            room = self.max_batch - len(active)
            new = feed.take(room, wait=not active) if room > 0 else []
            if not new and not active:
                if feed.done:
                    return
                continue
            self.stats["prefills"] += len(new)
            active += [[self.steps, item[0], item[1]] for item in new]
            time.sleep(self.step_s)
            self.stats["decode_steps"] += 1
            still = []
            for a in active:
                a[0] -= 1
                if a[0] > 0:
                    still.append(a)
                    continue
                inp = a[2]
                yield a[1], json.dumps({"description": f"{inp.full_class_name} (pid {os.getpid()})",
                                        "classTypeCorrection": None,
                                        "methods": [{"methodName": m, "description": "does " + m,
                                                     "businessLogic": ["step"]} for m in inp.method_names]})
            active = still


def _witness(dev: str) -> dict:
    """What this worker runs on, from the device itself (hipGetDeviceProperties)
    and the kernel library it loaded -- reported next to every throughput
    number the worker produces."""
    if not dev.startswith("cuda"):
        return {"device": dev}
    try:
        import torch
        p = torch.cuda.get_device_properties(0)
        out = {"name": p.name, "arch": getattr(p, "gcnArchName", ""), "cus": p.multi_processor_count,
               "hbm_gib": round(p.total_memory / 2**30, 1)}
        from ..ops import hip
        out["hipops"] = os.path.relpath(hip.TARGET if not os.environ.get("DMCP_HIPOPS_SO") else
                                        os.environ["DMCP_HIPOPS_SO"])
        out["hipops_abi"] = int(hip.lib().dmcp_abi_version())
        return out
    except Exception as e:  # noqa: BLE001 -- a witness, never a failure
        return {"device": dev, "error": repr(e)[:200]}


def worker_main() -> int:
    """``python -m dmcp.enrich.workers``: serve frames on stdin/stdout."""
    rx = sys.stdin.buffer
    tx = sys.stdout.buffer
    sys.stdout = sys.stderr  # nothing else may write to the protocol pipe
    logging.basicConfig(level=os.environ.get("LOG_LEVEL", "WARNING").upper(), stream=sys.stderr,
                        format="%(asctime)s [worker %(process)d] %(levelname)s %(name)s - %(message)s")
    txlock = threading.Lock()
    if os.environ.get("DMCP_WORKER_DEBUG"):
        import faulthandler
        faulthandler.dump_traceback_later(20, repeat=True, file=sys.stderr)

    def send(obj) -> None:
        with txlock:
            send_frame(tx, obj)

    msg = recv_frame(rx)
    if msg is None or msg.get("op") != "init":
        return 0 if msg is None or msg.get("op") == "shutdown" else 2
    spec = msg["model"]
    dev = msg.get("device", "cuda:0")
    from .feeds import MultiFeed
    if spec.get("preset") == "echo":
        eng = _EchoEngine(float(spec.get("step_s", 0.05)), int(spec.get("max_batch", 512)), int(spec.get("steps", 1)))
        max_batch = eng.max_batch
    else:
        import torch
        from .local import LocalEngine, build_model
        try:
            if dev.startswith("cuda"):
                torch.cuda.set_device(0)
            model, tok = build_model(spec, dev)
            eng = LocalEngine(model, tokenizer=tok, **(msg.get("engine") or {}))
        except Exception as e:
            send({"op": "error", "msg": f"init failed: {e!r}"})
            return 3
        max_batch = model.cfg.max_batch
    send({"op": "ready", "pid": os.getpid(), "device": dev,
          "gpu": os.environ.get("HIP_VISIBLE_DEVICES", ""), "max_batch": max_batch, "witness": _witness(dev)})

    # ONE engine stream over every session: the projects the pool deals this
    # worker share its continuous batch (MultiFeed: round-robin over them)
    feed = MultiFeed()
    lock = threading.Lock()
    outstanding: Dict[int, int] = {}        # sid -> classes received, reply not yet sent
    closed: set = set()                     # sids whose ``end`` arrived
    base: Dict[int, Dict[str, float]] = {}  # sid -> engine stats at its begin

    def finish(sid: int) -> None:  # caller holds ``lock``
        if sid in closed and outstanding.get(sid, 0) == 0:
            st = {k: v - base.get(sid, {}).get(k, 0) for k, v in eng.stats.items() if isinstance(v, (int, float))}
            outstanding.pop(sid, None)
            closed.discard(sid)
            base.pop(sid, None)
            send({"op": "done", "sid": sid, "stats": st})

    def reader() -> None:
        while True:
            m = recv_frame(rx)
            if m is None or m.get("op") == "shutdown":
                feed.shutdown()
                return
            op, sid = m.get("op"), m.get("sid")
            with lock:
                if op == "begin":
                    outstanding[sid] = 0
                    base[sid] = dict(eng.stats)
                    feed.begin(sid, m.get("readme"))
                elif op == "items" and sid in outstanding:
                    outstanding[sid] += len(m["items"])
                    feed.put(sid, [(k, _inp_from_wire(v)) for k, v in m["items"]])
                elif op == "end" and sid in outstanding:
                    closed.add(sid)
                    feed.end(sid)
                    finish(sid)

    threading.Thread(target=reader, name="rx", daemon=True).start()
    try:
        for (sid, key), raw in eng.stream(feed, None):
            send({"op": "result", "sid": sid, "items": [[key, raw]]})
            with lock:
                if sid in outstanding:
                    outstanding[sid] -= 1
                finish(sid)
    except Exception as e:  # a GPU-touched process is not reused after a failure
        LOG.exception("engine failed")
        send({"op": "error", "msg": repr(e)})
        return 4
    return 0


if __name__ == "__main__":
    raise SystemExit(worker_main())
