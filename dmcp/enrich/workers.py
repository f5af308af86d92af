"""One worker process per GPU for the local enrichment model -- MI355X extension.

Enrichment requests are independent (one prompt per class,
``ClaudeApiClient.java:288-329``), so multi-GPU scaling is pure data
parallelism: every MI355X holds a full copy of the model and
its own KV-cache slab, and classes are handed out from ONE queue in the
parent.  Each replica lives in its own process:

* the parent (REST / MCP / CLI service) starts the workers BEFORE it touches
  HIP and never initialises the GPU itself -- each child sees exactly one
  device (``HIP_VISIBLE_DEVICES``), so a fault or hang on one GPU kills one
  child, never the server;
* each engine's ~0.3 ms of host work per decode step (grammar state machine,
  row packing) runs on its own interpreter -- N replicas driven by N threads
  of one process would serialise on the GIL (8 x 0.3 ms against a 2-4 ms
  step);
* parent and child talk over the child's stdin / stdout: length-prefixed
  JSON frames (``begin`` readme / ``items`` / ``end`` down; ``ready`` /
  ``result`` / ``done`` / ``error`` up); the child's logs go to stderr;
* the parent keeps every worker's queue ``max_batch * 1.5`` classes deep so
  its continuous batch never drains, yields each result as it arrives, and
  when a worker dies (EOF on its pipe, a non-zero exit, or no frame for
  ``hang_timeout_s`` while it holds work -- then it is killed) the classes it
  held are reported as failures (Phase 3 retries them) and the rest go to
  the live workers.  A dead worker is replaced by a FRESH child at the next
  stream; a GPU-touched process is never restarted in place.
"""
from __future__ import annotations

import json
import logging
import os
import queue
import struct
import subprocess
import sys
import threading
import time
from typing import Any, Dict, Iterable, Iterator, List, Optional, Sequence, Tuple

from .backend import EnrichmentBackend
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
    def __init__(self, index: int, device: str, events: "queue.Queue", env_extra: Optional[dict] = None) -> None:
        self.index = index
        self.device = device  # "cuda:<physical id>" or "cpu"
        self.events = events
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
        self.ready = False
        self.info: dict = {}
        self.inflight: Dict[int, str] = {}   # key -> class name
        self.last_frame = time.monotonic()
        self.done_sid = 0
        self.stats: Dict[str, float] = {}
        self.sent = 0
        self._wlock = threading.Lock()
        self._reader = threading.Thread(target=self._read, name=f"gpu-worker-{index}-rx", daemon=True)
        self._reader.start()

    def _read(self) -> None:
        out = self.proc.stdout
        while True:
            try:
                msg = recv_frame(out)
            except Exception as e:  # corrupt frame: treat as death
                LOG.error("worker %d: bad frame: %s", self.index, e)
                msg = None
            # tagged with this worker object, not its index: a replaced
            # worker's late EOF must not mark its successor dead
            self.events.put((self, msg))
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


class GpuWorkerPool:
    """N worker processes, one per device; :meth:`stream` runs one enrichment
    stream across all of them.  Spawn (cheap: the children import nothing
    heavy until ``init``) before this process touches HIP."""

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
        self.events: "queue.Queue" = queue.Queue()
        self.workers: List[_Worker] = [self._spawn(i) for i in range(len(self.devices))]
        self.sid = 0
        self.deaths = 0
        self.per_worker_items: Dict[int, int] = {}
        self._lock = threading.Lock()
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
        return _Worker(i, self.devices[i], self.events, extra)

    @property
    def capacity(self) -> int:
        mb = int(self.model.get("max_batch", 256))
        return mb + max(2, mb // 2)

    def init(self) -> None:
        """Builds the model in every worker (in parallel); waits for all."""
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
                who, msg = self.events.get(timeout=min(1.0, left))
            except queue.Empty:
                continue
            if self._current(who):
                self._handle_control(who.index, msg)
        if not any(w.ready for w in self.workers):
            raise RuntimeError("no GPU worker started")
        self._initialised = True

    def _current(self, w: "_Worker") -> bool:
        """False for events of a worker that was already replaced."""
        return 0 <= w.index < len(self.workers) and self.workers[w.index] is w

    def _handle_control(self, i: int, msg: Optional[dict]) -> None:
        w = self.workers[i]
        if msg is None:
            if w.alive:
                LOG.error("worker %d on %s exited (rc=%s)", i, w.device, w.proc.poll())
            w.alive = False
            return
        w.last_frame = time.monotonic()
        if msg.get("op") == "ready":
            w.ready = True
            w.info = msg
            LOG.info("GPU worker %d ready on %s (pid %s)", i, w.device, msg.get("pid"))
        elif msg.get("op") == "error":
            LOG.error("worker %d: %s", i, msg.get("msg"))

    def _replace_dead(self) -> None:
        respawned = False
        for i, w in enumerate(self.workers):
            if not w.alive:
                w.kill()
                self.workers[i] = self._spawn(i)
                respawned = True
        if respawned:
            self.init()

    def stream(self, inputs: Iterable[EnrichmentInput], readme: Optional[str]
               ) -> Iterator[Tuple[int, Any]]:
        """Yields ``(input index, raw reply str | Exception)`` as replies
        arrive, from whichever worker finished them.  A caller that stops
        early (an exception while applying a reply) still ends the session
        in every worker: each finishes what it was sent and then serves the
        next stream (its late replies carry the old session id and are
        dropped)."""
        with self._lock:
            self._open: List[_Worker] = []
            try:
                yield from self._stream(inputs, readme)
            finally:
                for w in self._open:
                    if w.alive:
                        w.send({"op": "end", "sid": self.sid})
                self._open = []

    def _stream(self, inputs, readme):
        self._replace_dead()
        self.sid += 1
        sid = self.sid
        src = enumerate(inputs)
        exhausted = False
        live = [w for w in self.workers if w.alive and w.ready]
        for w in live:
            w.inflight.clear()
            if not w.send({"op": "begin", "sid": sid, "readme": readme}):
                w.alive = False
        ended: set = set()
        self._open = [w for w in live if w.alive]  # sessions to end if the caller stops early
        finished: set = set()
        cap = self.capacity
        chunk_min = max(1, cap // 8)

        def top_up(w: _Worker) -> None:
            nonlocal exhausted
            need = cap - len(w.inflight)
            if exhausted or need < (chunk_min if w.inflight else 1):
                return
            items = []
            while len(items) < need:
                try:
                    i, inp = next(src)
                except StopIteration:
                    exhausted = True
                    break
                items.append([i, _inp_to_wire(inp)])
                w.inflight[i] = inp.full_class_name
            if items:
                self.per_worker_items[w.index] = self.per_worker_items.get(w.index, 0) + len(items)
                w.sent += len(items)
                if not w.send({"op": "items", "sid": sid, "items": items}):
                    w.alive = False

        def fail(w: _Worker, why: str):
            for k, name in list(w.inflight.items()):
                yield k, RuntimeError(f"{why} (worker {w.index} on {w.device})")
            w.inflight.clear()

        while True:
            live = [w for w in self.workers if w.alive and w.ready]
            for w in live:
                top_up(w)
            for w in list(self.workers):
                if not w.alive and w.inflight:
                    self.deaths += 1
                    yield from fail(w, "GPU worker died")
            live = [w for w in self.workers if w.alive and w.ready]
            if not live:
                # nothing can run the rest: every remaining class fails
                for i, inp in src:
                    yield i, RuntimeError("no live GPU worker")
                return
            if exhausted:
                for w in live:
                    if w not in ended:
                        w.send({"op": "end", "sid": sid})
                        ended.add(w)
                        if w in self._open:
                            self._open.remove(w)
                if all(w in finished or not w.alive for w in self.workers if w in ended) and \
                        not any(w.inflight for w in self.workers):
                    return
            try:
                who, msg = self.events.get(timeout=1.0)
            except queue.Empty:
                now = time.monotonic()
                for w in live:
                    if w.inflight and now - w.last_frame > self.hang_timeout_s:
                        LOG.error("worker %d on %s sent nothing for %.0f s with %d classes: killing it", w.index,
                                  w.device, self.hang_timeout_s, len(w.inflight))
                        w.kill()
                continue
            if not self._current(who):
                continue
            w, i = who, who.index
            if msg is None:
                if w.alive:
                    LOG.error("worker %d on %s exited (rc=%s) holding %d classes", i, w.device, w.proc.poll(),
                              len(w.inflight))
                w.alive = False
                continue
            w.last_frame = time.monotonic()
            op = msg.get("op")
            if op == "result" and msg.get("sid") == sid:
                for k, raw in msg["items"]:
                    if w.inflight.pop(k, None) is not None:
                        yield k, raw
            elif op == "done" and msg.get("sid") == sid:
                w.stats = msg.get("stats") or {}
                finished.add(w)
            elif op == "error":
                LOG.error("worker %d on %s: %s", i, w.device, msg.get("msg"))
                w.kill()  # it exits on its own; never reused

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
    process per GPU) behind the :class:`EnrichmentBackend` contract."""

    name = "local"

    def __init__(self, pool: GpuWorkerPool) -> None:
        super().__init__(max_concurrent=1)
        self.pool = pool
        self.preferred_batch_size = pool.capacity * len(pool.workers)

    @classmethod
    def from_config(cls, cfg, devices: Optional[Sequence[str]] = None) -> "ProcessLLMBackend":
        if devices is None:
            n = visible_gpus()
            spec = (cfg.local_llm_devices or "all").strip()
            ids = list(range(n)) if spec == "all" else [int(x) for x in spec.split(",") if x.strip()]
            if not ids:
                raise RuntimeError("the local enrichment backend needs a ROCm GPU (none visible)")
            devices = [f"cuda:{d}" for d in ids]
        mb = int(cfg.local_llm_max_batch)
        model = {"preset": cfg.local_llm_preset, "kv_dtype": cfg.local_llm_kv_dtype, "max_batch": mb,
                 "max_rows": max(256, mb * 3 // 2), "seed": 0}
        if getattr(cfg, "local_llm_model_path", ""):
            model["path"] = cfg.local_llm_model_path
        return cls(GpuWorkerPool(devices, model))

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

        def tagged():
            for i, inp in enumerate(inputs):
                names[i] = inp.full_class_name
                yield inp
        for i, raw in self.pool.stream(tagged(), readme):
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


# ------------------------------------------------------------------ child
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
    import torch
    from .local import LocalEngine, QueueFeed, build_model
    spec = msg["model"]
    dev = msg.get("device", "cuda:0")
    try:
        if dev.startswith("cuda"):
            torch.cuda.set_device(0)
        model, tok = build_model(spec, dev)
        eng = LocalEngine(model, tokenizer=tok, **(msg.get("engine") or {}))
    except Exception as e:
        send({"op": "error", "msg": f"init failed: {e!r}"})
        return 3
    send({"op": "ready", "pid": os.getpid(), "device": dev,
          "gpu": os.environ.get("HIP_VISIBLE_DEVICES", ""), "max_batch": model.cfg.max_batch})

    sessions: "queue.Queue" = queue.Queue()
    feeds: Dict[int, QueueFeed] = {}

    def reader() -> None:
        while True:
            m = recv_frame(rx)
            if m is None or m.get("op") == "shutdown":
                for f in feeds.values():
                    f.close()
                sessions.put(None)
                return
            op = m.get("op")
            if op == "begin":
                f = QueueFeed()
                feeds[m["sid"]] = f
                sessions.put((m["sid"], m.get("readme"), f))
            elif op == "items":
                f = feeds.get(m["sid"])
                if f is not None:
                    f.put((k, _inp_from_wire(v)) for k, v in m["items"])
            elif op == "end":
                f = feeds.get(m["sid"])
                if f is not None:
                    f.close()

    threading.Thread(target=reader, name="rx", daemon=True).start()
    while True:
        s = sessions.get()
        if s is None:
            return 0
        sid, readme, feed = s
        for k in eng.stats:
            eng.stats[k] = 0
        try:
            for key, raw in eng.stream(feed, readme):
                send({"op": "result", "sid": sid, "items": [[key, raw]]})
        except Exception as e:  # a GPU-touched process is not reused after a failure
            LOG.exception("engine failed")
            send({"op": "error", "sid": sid, "msg": repr(e)})
            return 4
        feeds.pop(sid, None)
        send({"op": "done", "sid": sid, "stats": dict(eng.stats)})


if __name__ == "__main__":
    raise SystemExit(worker_main())
