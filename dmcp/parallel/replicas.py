"""Data-parallel replicas of the local enrichment model (one per GPU).

Enrichment requests are independent, so multi-GPU scaling is pure data
parallelism: every MI355X holds a full copy of the (small) model and its own
KV-cache slab, and classes are handed out from one shared queue
(work-stealing, so a replica that drew short replies takes more work).  There
is no collective in the hot path -- xGMI bandwidth is irrelevant to this
workload; each replica is driven by its own host thread, which
releases the GIL inside HIP calls.
"""
from __future__ import annotations

import logging
import threading
from typing import Callable, Dict, List, Optional, Sequence, Tuple

LOG = logging.getLogger(__name__)


class ReplicaPool:
    """Runs ``fn(replica, items)`` over chunks of a work list on every replica.

    ``chunk`` items are taken at a time (a replica's continuous batch is
    refilled as it drains); results come back in input order.  A failing
    chunk is reported per item through ``on_error`` and does not stop the
    other replicas.
    """

    def __init__(self, replicas: Sequence, chunk_for: Optional[Callable[[object], int]] = None) -> None:
        if not replicas:
            raise ValueError("ReplicaPool needs at least one replica")
        self.replicas = list(replicas)
        self.chunk_for = chunk_for or (lambda r: 64)
        self.stats: Dict[int, int] = {i: 0 for i in range(len(self.replicas))}

    def map(self, fn: Callable[[object, List], List], items: Sequence,
            on_error: Optional[Callable[[int, BaseException], object]] = None,
            device_ctx: Optional[Callable[[object], object]] = None) -> List:
        n = len(items)
        out: List = [None] * n
        nxt = [0]
        lock = threading.Lock()

        def take(k: int) -> Tuple[int, int]:
            with lock:
                a = nxt[0]
                b = min(n, a + k)
                nxt[0] = b
                return a, b

        def worker(ri: int) -> None:
            rep = self.replicas[ri]
            k = max(1, int(self.chunk_for(rep)))
            while True:
                a, b = take(k)
                if a >= b:
                    return
                try:
                    if device_ctx is not None:
                        with device_ctx(rep):
                            res = fn(rep, list(items[a:b]))
                    else:
                        res = fn(rep, list(items[a:b]))
                    if len(res) != b - a:
                        raise RuntimeError(f"replica {ri} returned {len(res)} results for {b - a} items")
                    out[a:b] = res
                    with lock:
                        self.stats[ri] += b - a
                except BaseException as e:  # isolate: this chunk fails, the rest continue
                    LOG.exception("replica %d failed on items [%d, %d)", ri, a, b)
                    for i in range(a, b):
                        out[i] = on_error(i, e) if on_error is not None else e

        if len(self.replicas) == 1:
            worker(0)
        else:
            threads = [threading.Thread(target=worker, args=(i,), name=f"replica-{i}")
                       for i in range(len(self.replicas))]
            for t in threads:
                t.start()
            for t in threads:
                t.join()
        return out
