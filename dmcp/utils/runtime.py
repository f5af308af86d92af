"""Process-level runtime tuning.

CPython's cyclic GC walks every tracked object on each generation-2 pass.  A
service process that has imported PyTorch (the local-enrichment backend, the
benchmark's RCCL plumbing) carries ~10^6 long-lived objects, so the frequent
collections triggered by the indexer's many short-lived rows became the
largest cost of an analysis: measured on an MI355X host, one 2,000-class
analysis took 184 ms without torch imported and 300 ms with it; with the
start-up heap frozen and a larger gen-0 threshold it is back to 191 ms.

Inside one analysis the remaining cost is a single generation-0 pass over the
analysis' own young objects (parsed units, graph nodes, Phase-1 rows: ~50k
at 2,000 classes), which lands wherever the allocation count crosses the
threshold -- usually in Phase 1, on the main thread's critical path
(5-12 ms; ``analyze.phase1`` 5.6 ms on runs it missed, 11-23 ms on runs it
hit).  :class:`GcPause` holds the automatic passes off for that burst and
runs the one young pass later, where the main thread waits for the native
row writer anyway (its thread holds no GIL).
"""
from __future__ import annotations

import gc
import threading

_tuned = False
_lock = threading.Lock()

GEN0_THRESHOLD = 50_000


def tune_gc() -> None:
    """Freeze the objects alive now (imports, configuration, caches) out of
    the cyclic collector and raise the gen-0 threshold.  Idempotent; call
    after start-up imports."""
    global _tuned
    with _lock:
        gc.freeze()
        if not _tuned:
            _, g1, g2 = gc.get_threshold()
            gc.set_threshold(GEN0_THRESHOLD, max(g1, 20), max(g2, 20))
            _tuned = True


_pause_lock = threading.Lock()
_pauses = 0          # GcPause sections open in this process (any thread)
_was_enabled = False  # the collector's state when the first one opened


class GcPause:
    """Automatic cyclic-GC passes held off from :meth:`start` to
    :meth:`resume` (process-wide: the collector has one switch; sections on
    several threads nest by count and the last one out restores the state
    the first one found).  The objects allocated meanwhile are freed by
    reference counting as usual; only cycles wait for the next pass.
    ``resume(collect=True)`` runs the deferred generation-0 pass right away,
    when there is one to run.  Idempotent; safe in ``finally``."""

    def __init__(self) -> None:
        self.active = False

    def start(self) -> "GcPause":
        global _pauses, _was_enabled
        with _pause_lock:
            if not self.active:
                if _pauses == 0:
                    _was_enabled = gc.isenabled()
                    gc.disable()
                _pauses += 1
                self.active = True
        return self

    def resume(self, collect: bool = False) -> None:
        global _pauses
        with _pause_lock:
            if not self.active:
                return
            self.active = False
            _pauses -= 1
            if _pauses > 0 or not _was_enabled:
                return
            gc.enable()
        if collect and gc.get_count()[0] >= gc.get_threshold()[0]:
            gc.collect(0)

    def __enter__(self) -> "GcPause":
        return self.start()

    def __exit__(self, *exc) -> None:
        self.resume()
