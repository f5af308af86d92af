"""Process-level runtime tuning.

CPython's cyclic GC walks every tracked object on each generation-2 pass.  A
service process that has imported PyTorch (the local-enrichment backend, the
benchmark's RCCL plumbing) carries ~10^6 long-lived objects, so the frequent
collections triggered by the indexer's many short-lived rows became the
largest cost of an analysis: measured on an MI355X host, one 2,000-class
analysis took 184 ms without torch imported and 300 ms with it; with the
start-up heap frozen and a larger gen-0 threshold it is back to 191 ms.
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
